#!/usr/bin/env python3
"""Device decrypt only (K ciphertexts of one cfg3 learner, 2^15 / L4, exact decode), for
rocprofv3 kernel stats of diagnostic decrypt variants: python tools/dec_time.py [K] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 714
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7, decodeNoise=False)
assert ck.genCryptoContextAndKeyGen() == 1
x = torch.rand(K * 16384, device="cuda", dtype=torch.float64) * 2 - 1
ct = D.encrypt(ck, x)
out = D.decrypt(ck, ct, K * 16384, ck.info()["delta"])
for _ in range(reps):
    D.decrypt(ck, ct, K * 16384, ck.info()["delta"], out=out)
torch.cuda.synchronize()
print("ok")
