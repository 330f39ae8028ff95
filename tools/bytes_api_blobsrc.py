#!/usr/bin/env python3
"""Does the bytes API's aggregation rate depend on where the learners' blobs came from (round 5: bench's
archive sample ran 31-46 GB/s while tools/bytes_api_ab.py measured 52 for the same call)?  Encrypt outputs
as they are, the same bytes copied into fresh objects, and both again after the process has allocated a
cfg3-sized device arena and device encrypts (what bench does first).  Median of 5 calls each, results kept.
    python tools/bytes_api_blobsrc.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402  (before the library touches the GPU)

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

Cl, Ka, B = 16, 64, 16384
d = "/tmp/keys_bytes_src/"
os.makedirs(d, exist_ok=True)
ck = m.CKKS("ckks", B, 52, d, multDepth=3, seed=7)
assert ck.genCryptoContextAndKeyGen() == 1
w = [1.0 / Cl] * Cl
out = {}


def rate(blobs):
    ck.computeWeightedAverage(blobs, w)
    kept, ts = [], []
    for _ in range(5):
        t0 = time.perf_counter()
        kept.append(ck.computeWeightedAverage(blobs, w))
        ts.append(time.perf_counter() - t0)
    dt = sorted(ts)[2]
    return round(sum(len(b) for b in blobs) / dt / 1e9, 2)


x = np.random.default_rng(1).uniform(-1, 1, Ka * B)
enc = [ck.encrypt(x) for _ in range(Cl)]
out["encrypt_outputs"] = rate(enc)
out["fresh_copies"] = rate([bytes(bytearray(b)) for b in enc])
print(json.dumps(out), flush=True)
K = 714
xs = torch.rand(K * B, device="cuda", dtype=torch.float64) * 2 - 1
cts = [D.encrypt(ck, xs) for _ in range(4)]
ar = D.Arena(ck, 16, K, layout="packed")
for i in range(16):
    ar.put(i, cts[i % 4])
torch.cuda.synchronize()
out["encrypt_outputs_after_arena"] = rate(enc)
enc2 = [ck.encrypt(x) for _ in range(Cl)]
out["new_encrypt_outputs_after_arena"] = rate(enc2)
out["fresh_copies_after_arena"] = rate([bytes(bytearray(b)) for b in enc2])
print(json.dumps(out), flush=True)
# what bench does before its API sample: per learner, a float32 host vector copied to the device
for i in range(16):
    xh = np.random.default_rng(1000 + i).uniform(-1, 1, K * B).astype(np.float32)
    t = torch.from_numpy(xh).to("cuda").double()
    del xh, t
torch.cuda.synchronize()
out["encrypt_outputs_after_host_uploads"] = rate(enc2)
enc3 = [ck.encrypt(x) for _ in range(Cl)]
out["new_encrypt_outputs_after_host_uploads"] = rate(enc3)
print(json.dumps({"what": "bytes-API wavg input GB/s, 16 x 64 cts PALISADE archives, median of 5", **out}))
