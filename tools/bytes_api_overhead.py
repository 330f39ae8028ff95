#!/usr/bin/env python3
"""Where the bytes-API aggregation's time goes outside its upload pipeline (round 5): the sizing call
(parses every learner's blob, no device work), the output bytes allocation, and the whole call, on warm
blobs, median of 7.  SHELFI_STAGE_TRACE=1 adds the pipeline's own issue / tail split on stderr.
    python tools/bytes_api_overhead.py [--wire palisade]"""
import argparse
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

ap = argparse.ArgumentParser()
ap.add_argument("--wire", default="palisade")
ap.add_argument("--cts", type=int, default=64, help="ciphertexts per learner (cfg2: 4)")
a = ap.parse_args()
Cl, Ka, B = 16, a.cts, 16384
d = "/tmp/keys_bytes_ovh/"
os.makedirs(d, exist_ok=True)
ck = m.CKKS("ckks", B, 52, d, multDepth=3, seed=7)
assert ck.genCryptoContextAndKeyGen() == 1
ck.set_wire_format(a.wire)
w = [1.0 / Cl] * Cl
x = np.random.default_rng(1).uniform(-1, 1, Ka * B)
blobs = [ck.encrypt(x) for _ in range(Cl)]
nb = sum(len(b) for b in blobs)
ck.computeWeightedAverage(blobs, w)
arr = (_lib.u8p * Cl)()
lens = (C.c_size_t * Cl)()
for i, b in enumerate(blobs):
    arr[i] = C.cast(C.c_char_p(b), _lib.u8p)
    lens[i] = len(b)
wf = np.asarray(w, dtype=np.float32)
wp = wf.ctypes.data_as(_lib.f32p)
n_out = C.c_size_t()


def med(f, n=7):
    ts = []
    kept = []
    for _ in range(n):
        t0 = time.perf_counter()
        kept.append(f())
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[n // 2] * 1e3


res = {
    "sizing_call_ms": med(lambda: ck._lib.shelfi_weighted_average_into(ck._ctx, arr, lens, wp, Cl, None, 0, C.byref(n_out))),
    "new_bytes_ms": med(lambda: m._new_bytes(n_out.value)),
    "whole_call_ms": med(lambda: ck.computeWeightedAverage(blobs, w), 15 if Ka < 16 else 7),
}
res["input_GB_per_s"] = round(nb / res["whole_call_ms"] / 1e6, 2)
print(json.dumps({"what": "bytes-API aggregation outside the pipeline, %s wire, 16 x %d cts, warm, median" % (a.wire, Ka),
                  **{k: round(v, 3) for k, v in res.items()}}))
