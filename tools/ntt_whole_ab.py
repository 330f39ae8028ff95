#!/usr/bin/env python3
"""Round 6 A/B for VERDICT r5 item 3: the whole-polynomial forward NTT probe
(tools/ntt_whole_probe.hip: one 1024-thread workgroup per 2^15 polynomial, 32 residues per
thread, LDS transposes) against the library's two-pass NTT (shelfi_dev_ntt = launch_ntt:
ntt_fwd_cols<4> + ntt_fwd_blocks_ct<11, ...> through HBM) on the same polynomials in one
process, alternated, outputs compared bit for bit; and the device encrypt of the same learner
(K ciphertexts = 3 L K NTTs, plus sampling, encode and the key combine) as the per-NTT budget
a fused whole-polynomial encrypt would have to beat.

  python tools/ntt_whole_ab.py [K] [reps]       (K = 714: a cfg3 learner, 8,568 NTTs)

Build (once, on the CPU): hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950
  -ffp-contract=off -o tools/ntt_whole_probe.so tools/ntt_whole_probe.hip"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

LOGN = 15
N = 1 << LOGN
NORED_Q = 1 << 57


def bitrev(n_bits):
    i = np.arange(1 << n_bits, dtype=np.uint64)
    r = np.zeros_like(i)
    for b in range(n_bits):
        r |= ((i >> np.uint64(b)) & np.uint64(1)) << np.uint64(n_bits - 1 - b)
    return r


def tables(moduli, roots):
    """psi_rev[i] = psi^bitrev(i) with Shoup companions, [L][N][2]; tower constants [L][4]."""
    L = len(moduli)
    br = bitrev(LOGN)
    tw = np.zeros((L, N, 2), np.uint64)
    tq = np.zeros((L, 4), np.uint64)
    for t, (q, psi) in enumerate(zip(moduli, roots)):
        pw = [1] * N
        for i in range(1, N):
            pw[i] = pw[i - 1] * psi % q
        W = [pw[int(b)] for b in br]
        tw[t, :, 0] = np.array(W, dtype=np.uint64)
        tw[t, :, 1] = np.array([(w << 64) // q for w in W], dtype=np.uint64)
        tq[t] = [q, (1 << 64) - 8 * q, (1 << 64) // q, 0]
    return tw, tq


def tower_runs(moduli):
    """consecutive tower ranges of one class: (t0, nt, nored)"""
    runs = []
    for t, q in enumerate(moduli):
        nr = int(q < NORED_Q)
        if runs and runs[-1][2] == nr:
            runs[-1][1] += 1
        else:
            runs.append([t, 1, nr])
    return runs


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 714
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    probe = C.CDLL(os.path.join(ROOT, "tools", "ntt_whole_probe.so"))
    probe.ntt_whole_fwd.restype = C.c_int
    probe.ntt_whole_fwd.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                    C.c_void_p, C.c_void_p, C.c_void_p]
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    assert inf["ring_dim"] == N
    L, moduli, roots = inf["num_towers"], inf["moduli"], inf["roots"]
    tw_h, tq_h = tables(moduli, roots)
    dev = torch.device("cuda")
    tw = torch.from_numpy(tw_h.view(np.int64)).to(dev)
    tq = torch.from_numpy(tq_h.view(np.int64)).to(dev)
    runs = tower_runs(moduli)
    P = 3 * K * L
    g = torch.Generator(device=dev).manual_seed(11)
    X = torch.empty((3 * K, L, N), dtype=torch.int64, device=dev)
    for t, q in enumerate(moduli):
        X[:, t, :] = torch.randint(0, q, (3 * K, N), generator=g, device=dev, dtype=torch.int64)
    A = torch.empty_like(X)
    B = torch.empty_like(X)
    stream = torch.cuda.current_stream()

    def whole(buf):
        for t0, nt, nr in runs:
            rc = probe.ntt_whole_fwd(C.c_void_p(buf.data_ptr()), P, L, t0, nt, nr, C.c_void_p(tw.data_ptr()),
                                     C.c_void_p(tq.data_ptr()), C.c_void_p(stream.cuda_stream))
            assert rc == 0, rc

    def two_pass(buf):
        D.ntt(ck, buf.view(P, N))

    A.copy_(X)
    two_pass(A)
    B.copy_(X)
    whole(B)
    torch.cuda.synchronize()
    exact = bool(torch.equal(A, B))
    times = {"two_pass": [], "whole": []}
    for _ in range(reps):
        for name, fn, buf in (("two_pass", two_pass, A), ("whole", whole, B)):
            buf.copy_(X)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn(buf)
            e1.record(stream)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1e3)  # us
    # the device encrypt of K ciphertexts: 3 L K NTTs plus the rest of the chain
    B_ = inf["batch"]
    x = torch.rand(K * B_, generator=g, device=dev, dtype=torch.float64) * 2 - 1
    out = D.encrypt(ck, x)
    torch.cuda.synchronize()
    enc = []
    for _ in range(reps):
        t0 = time.perf_counter()
        D.encrypt(ck, x, out=out)
        torch.cuda.synchronize()
        enc.append((time.perf_counter() - t0) * 1e6)
    med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
    enc_us = sorted(enc)[len(enc) // 2]
    res = {
        "K": K, "polys": P, "towers": L, "tower_runs": runs, "bit_exact_vs_launch_ntt": exact,
        "two_pass_us": med["two_pass"], "whole_us": med["whole"],
        "two_pass_us_per_ntt": med["two_pass"] / P, "whole_us_per_ntt": med["whole"] / P,
        "whole_over_two_pass": med["whole"] / med["two_pass"],
        "encrypt_us_per_ct": enc_us / K, "encrypt_us_per_ntt_budget": enc_us / P,
        "whole_ntts_only_over_encrypt": med["whole"] / enc_us,
        "samples": times, "encrypt_samples_us": enc,
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
