#!/usr/bin/env python3
"""Decrypt time (K = 714, 2^15 / L4) of the same ciphertexts in different buffers: the
encrypt output, a clone made after a 22 GiB allocation (bench.py's arena), and the
original again — does physical placement move decrypt like it moves wavg?"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

K = 714
ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7, decodeNoise=False)
assert ck.genCryptoContextAndKeyGen() == 1
inf = ck.info()
x = torch.rand(K * 16384, device="cuda", dtype=torch.float64) * 2 - 1
ct = D.encrypt(ck, x)


def t_dec(c, flood=False, reps=5):
    ck.set_decode_noise(flood)
    out = D.decrypt(ck, c, K * 16384, inf["delta"])
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        D.decrypt(ck, c, K * 16384, inf["delta"], out=out)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[reps // 2] * 1e6 / K


print("encrypt output      : %.3f us/ct (flooded %.3f)" % (t_dec(ct), t_dec(ct, True)))
big = torch.empty(22 << 30, dtype=torch.uint8, device="cuda")
c2 = ct.clone()
print("clone after 22 GiB  : %.3f us/ct (flooded %.3f)" % (t_dec(c2), t_dec(c2, True)))
print("encrypt output again: %.3f us/ct (flooded %.3f)" % (t_dec(ct), t_dec(ct, True)))
