"""The encrypt sampler stream v2 (round 3): the C oracle's or_sample_encrypt
against an independent pure-Python restatement on top of the RFC 8439-checked ChaCha20
block (test_oracle_kat.py), plus distribution checks.

v: 16 ternary samples per 128 stream bits (the base-3 digits of U / 2^128), e0 / e1: one
32-bit word per sample, the 63-bit CDT comparison completed by a tie word only when the top
31 bits tie.  The product defines this stream (PALISADE's own is a seeded BLAKE2 generator
that cannot be reproduced); the GPU kernels are checked against the oracle bit for bit in
test_gpu_parity.py / test_gpu_shapes.py."""
import numpy as np
import pytest

import oracle as O


def _key(seed):
    key = np.zeros(8, np.uint32)
    O.lib.or_seed_to_key(seed, O._p(key, O.u32p))
    return key


def _py_sample(seed, g, N):
    """Pure-Python v2 stream: Python integers for the 128-bit digits and the 63-bit CDT."""
    key = _key(seed)
    cdt = [int(x) for x in O.gauss_cdt()]
    nonce = (1 << 56) | g
    N16, V0 = N // 16, N // 64
    v = np.zeros(N, np.int64)
    e0 = np.zeros(N, np.int64)
    e1 = np.zeros(N, np.int64)

    def blk(b):
        return [int(x) for x in O.chacha20_block(key, b, nonce)]

    def gauss(w, lo):
        u = ((w >> 1) << 32) | lo
        k = sum(1 for c in cdt if u >= c)
        return -k if w & 1 else k

    for h in range(N16):
        vb, b0, b1, t0, t1 = blk(h // 4), blk(V0 + h), blk(V0 + N16 + h), blk(V0 + 2 * N16 + h), blk(V0 + 3 * N16 + h)
        w4 = vb[4 * (h % 4): 4 * (h % 4) + 4]
        U = w4[0] | (w4[1] << 32) | (w4[2] << 64) | (w4[3] << 96)
        for i in range(16):
            U *= 3
            digit, U = U >> 128, U & ((1 << 128) - 1)
            j = h + N16 * i
            v[j] = digit - 1
            e0[j] = gauss(b0[i], t0[i])
            e1[j] = gauss(b1[i], t1[i])
    return v, e0, e1


@pytest.mark.parametrize("N,g", [(1024, 0), (1024, 77), (2048, 5)])
def test_oracle_sampler_matches_python_restatement(N, g):
    got = O.sample_encrypt(42, g, N)
    exp = _py_sample(42, g, N)
    for a, b in zip(got, exp):
        assert np.array_equal(a, b)


def test_ternary_digits_are_uniform_and_sign_balanced():
    vs, es = [], []
    for g in range(8):
        v, e0, e1 = O.sample_encrypt(7, g, 8192)
        vs.append(v)
        es += [e0, e1]
    v = np.concatenate(vs)
    counts = np.bincount(v + 1, minlength=3) / v.size
    assert np.abs(counts - 1 / 3).max() < 0.01
    e = np.concatenate(es)
    assert abs(e.mean()) < 0.05 and abs(e.std() - 3.19) < 0.05
    assert np.abs(e).max() < 13 * 3.19
    # digits within a 128-bit group are not correlated at lag 1 (successive rows i, i + 1)
    v2 = vs[0].reshape(16, -1)
    c = np.corrcoef(v2[:-1].ravel(), v2[1:].ravel())[0, 1]
    assert abs(c) < 0.02
