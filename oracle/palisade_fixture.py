"""Test-only reader for the PALISADE 1.11 cereal-binary files the reference commits.

TEST INFRASTRUCTURE ONLY (see oracle/oracle.py header).  This is an independent
second reader used to check the product's own PALISADE reader
(fhe-fed_amd/csrc/palisade_io.cpp); it does not share code with it.

Files: ``code/resources/cryptoparams/{cryptocontext,key-public,key-private}.txt``
written by ``ckks.cpp:41,48,53`` (Serial::SerializeToFile, SerType::BINARY) and
the ciphertext dump ``code/mkhe/build/CT1.txt``.  Layout facts recovered offline
(SURVEY App. A):
  * every NativeVector is ``u64 len | len x u64 residues | u64 modulus``;
  * the context holds per tower ``u32 cyclotomic order | u32 ring dim | ... |
    u64 modulus | u64 root-of-unity``.
"""
from __future__ import annotations

import struct

import numpy as np


def _is_prime(n: int) -> bool:
    if n < 2:
        return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def read_context(path: str):
    """-> dict(N, q=[...], psi=[...]) from a PALISADE cryptocontext.txt."""
    data = open(path, "rb").read()
    towers = []
    seen = set()
    for off in range(0, len(data) - 16):
        M, N = struct.unpack_from("<II", data, off)
        if N < 1024 or N > (1 << 17) or N & (N - 1) or M != 2 * N:
            continue
        for g in range(0, 12):
            p = off + 8 + g
            if p + 16 > len(data):
                break
            q, psi = struct.unpack_from("<QQ", data, p)
            if q < (1 << 20) or q >= (1 << 62) or q % M != 1 or q in seen:
                continue
            if not _is_prime(q) or pow(psi, N, q) != q - 1:
                continue
            towers.append((off, N, q, psi))
            seen.add(q)
            break
    if not towers:
        raise ValueError("no towers found in %s" % path)
    N = towers[0][1]
    return {"N": N, "q": [t[2] for t in towers], "psi": [t[3] for t in towers],
            "offsets": [t[0] for t in towers]}


def read_vectors(path: str, N: int, moduli):
    """All NativeVectors of length N whose trailing modulus is in ``moduli``,
    in file order -> list of (offset, modulus, np.uint64 array)."""
    data = open(path, "rb").read()
    pat = struct.pack("<Q", N)
    mods = set(int(m) for m in moduli)
    out = []
    pos = 0
    while True:
        off = data.find(pat, pos)
        if off < 0:
            break
        start = off + 8
        end = start + 8 * N
        if end + 8 <= len(data):
            (mod,) = struct.unpack_from("<Q", data, end)
            if mod in mods:
                vals = np.frombuffer(data, dtype="<u8", count=N, offset=start).astype(np.uint64)
                if (vals < np.uint64(mod)).all():
                    out.append((start, mod, vals.copy()))
                    pos = end + 8
                    continue
        pos = off + 1
    return out


def read_keys(cryptodir: str):
    """-> (ctx, pk[2][L][N] (b, a), sk[L][N]) in EVALUATION domain."""
    ctx = read_context(cryptodir + "cryptocontext.txt")
    N, q = ctx["N"], ctx["q"]
    L = len(q)
    pv = read_vectors(cryptodir + "key-public.txt", N, q)
    sv = read_vectors(cryptodir + "key-private.txt", N, q)
    if len(pv) != 2 * L or len(sv) != L:
        raise ValueError("unexpected key layout: %d pk / %d sk vectors" % (len(pv), len(sv)))
    for i, (_, mod, _) in enumerate(pv):
        assert mod == q[i % L], "pk tower order"
    for i, (_, mod, _) in enumerate(sv):
        assert mod == q[i], "sk tower order"
    pk = np.stack([v for _, _, v in pv]).reshape(2, L, N)
    sk = np.stack([v for _, _, v in sv]).reshape(L, N)
    return ctx, pk, sk


def read_ciphertext_meta(path: str, N: int, moduli):
    """Metadata trailer of a serialized Ciphertext<DCRTPoly> (CT1.txt):
    after the last element vector: depth, level, scaling factor (f64), encoding."""
    vecs = read_vectors(path, N, moduli)
    data = open(path, "rb").read()
    last_end = vecs[-1][0] + 8 * N + 8
    tail = data[last_end:]
    return vecs, tail
