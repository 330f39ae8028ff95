#!/usr/bin/env python3
"""Counters of a slow and a fast (arena, output) pair (round 5; run under rocprofv3 --pmc): one cfg3-shard
packed arena, 8 candidate output buffers timed once (2 launches each), then 5 launches into the fastest
and 5 into the slowest.  The last 10 wavg_packed dispatches of the trace are therefore fast x5, slow x5.
Prints the candidates' times and the chosen pair.
    rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum --kernel-trace -- python3 tools/placement_pmc.py"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import _lib  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

K, Cn, B = 714, 16, 16384
ck = m.CKKS("ckks", B, 52, "", multDepth=3, seed=7, decodeNoise=False)
assert ck.genCryptoContextAndKeyGen() == 1
inf = ck.info()
L, N = inf["num_towers"], inf["ring_dim"]
x = torch.rand(K * B, device="cuda", dtype=torch.float64) * 2 - 1
ct = D.encrypt(ck, x)
del x
arena = D.Arena(ck, Cn, K, layout="packed")
for i in range(Cn):
    arena.put(i, ct)
del ct
w = [1.0 / Cn] * Cn
cands = [torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda") for _ in range(8)]
ms = []
for o in cands:
    arena.wavg(w, out=o)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    arena.wavg(w, out=o)
    e1.record()
    torch.cuda.synchronize()
    ms.append(round(e0.elapsed_time(e1), 4))
fast, slow = ms.index(min(ms)), ms.index(max(ms))
for idx in (fast, slow):
    for _ in range(5):
        arena.wavg(w, out=cands[idx])
    torch.cuda.synchronize()
print(json.dumps({"candidate_ms": ms, "fast": fast, "slow": slow, "order": "last 10 wavg dispatches: fast x5, slow x5"}))
