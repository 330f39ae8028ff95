#!/usr/bin/env python3
"""Where the bytes API's aggregation call spends its host time outside the upload pipeline (round 5):
the size query (archive parsing), the result's allocation, the whole call, and freeing the result, for 16
learners x 64 cts at 2^15 / L4 in the default (PALISADE) wire.  SHELFI_STAGE_TRACE=1 adds the pipeline's
own split.  Prints one JSON line (medians of 5).
    python tools/bytes_api_split.py"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import numpy as np  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import _lib  # noqa: E402

import argparse  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=64)
ap.add_argument("--wire", default="palisade")
a = ap.parse_args()
Cl, Ka, B = 16, a.k, 16384
d = "/tmp/keys_bytes_split/"
os.makedirs(d, exist_ok=True)
ck = m.CKKS("ckks", B, 52, d, multDepth=3, seed=7)
assert ck.genCryptoContextAndKeyGen() == 1
ck.set_wire_format(a.wire)
x = np.random.default_rng(1).uniform(-1, 1, Ka * B)
blobs = [ck.encrypt(x) for _ in range(Cl)]
w = np.full(Cl, 1.0 / Cl, np.float32)
arr = (_lib.u8p * Cl)()
lens = (C.c_size_t * Cl)()
for i, b in enumerate(blobs):
    arr[i] = C.cast(C.c_char_p(b), _lib.u8p)
    lens[i] = len(b)
wp = w.ctypes.data_as(_lib.f32p)
lib = ck._lib
res = {"size_query": [], "new_bytes": [], "into": [], "free": [], "full": []}
for _ in range(6):
    n_out = C.c_size_t()
    t0 = time.perf_counter()
    _lib.check(lib.shelfi_weighted_average_into(ck._ctx, arr, lens, wp, Cl, None, 0, C.byref(n_out)), "size")
    t1 = time.perf_counter()
    out = m._new_bytes(n_out.value)
    t2 = time.perf_counter()
    _lib.check(lib.shelfi_weighted_average_into(ck._ctx, arr, lens, wp, Cl, m._bytes_ptr(out), n_out.value,
                                                C.byref(n_out)), "into")
    t3 = time.perf_counter()
    del out
    t4 = time.perf_counter()
    r = ck.computeWeightedAverage(blobs, list(w))
    t5 = time.perf_counter()
    del r
    for k, v in (("size_query", t1 - t0), ("new_bytes", t2 - t1), ("into", t3 - t2), ("free", t4 - t3),
                 ("full", t5 - t4)):
        res[k].append(v * 1e3)
print(json.dumps({"what": "ms, median of 6 (first included)", "k": Ka, "wire": a.wire, **{k: round(sorted(v)[len(v) // 2], 3) for k, v in res.items()},
                  "in_MB": round(sum(len(b) for b in blobs) / 1e6, 1)}))
