#!/usr/bin/env python3
"""Bytes-API aggregation on COLD blobs (round 5): every timed call gets learner blobs in freshly allocated
memory, as an aggregator does when each round's uploads arrive (benchmark.py encrypts, then aggregates
every key once).  Fresh blobs of two kinds: new encrypt outputs (the library's own MADV_HUGEPAGE'd output)
and plain copies (bytes(bytearray(b)): malloc'd pages, like data off the network).  Settings are switch
sets re-read per call, alternated; the blob creation is outside the clock.
    python tools/bytes_api_cold.py [--rounds 4] base SHELFI_H2D_DIRECT=0 ..."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import numpy as np  # noqa: E402

import SHELFI_FHE as m  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--k", type=int, default=64)
ap.add_argument("--learners", type=int, default=16)
ap.add_argument("--wire", default="palisade")
ap.add_argument("settings", nargs="+")
a = ap.parse_args()
Cl, Ka, B = a.learners, a.k, 16384
d = "/tmp/keys_bytes_cold/"
os.makedirs(d, exist_ok=True)
ck = m.CKKS("ckks", B, 52, d, multDepth=3, seed=7)
assert ck.genCryptoContextAndKeyGen() == 1
ck.set_wire_format(a.wire)
w = [1.0 / Cl] * Cl
x = np.random.default_rng(1).uniform(-1, 1, Ka * B)
src = [ck.encrypt(x) for _ in range(Cl)]
nb = sum(len(b) for b in src)
keys = sorted({kv.split("=")[0] for st in a.settings if st != "base" for kv in st.split(",")})


def apply(st):
    for k in keys:
        os.environ.pop(k, None)
    if st != "base":
        for kv in st.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
    m.reload_switches()


ck.computeWeightedAverage(src, w)  # library buffers allocated
res = {st: {"encrypt_outputs": [], "copies": [], "warm": []} for st in a.settings}
for r in range(a.rounds):
    for st in (a.settings if r % 2 == 0 else a.settings[::-1]):
        apply(st)
        for kind in ("encrypt_outputs", "copies"):
            blobs = [ck.encrypt(x) for _ in range(Cl)] if kind == "encrypt_outputs" else [bytes(bytearray(b)) for b in src]
            t0 = time.perf_counter()
            out = ck.computeWeightedAverage(blobs, w)
            res[st][kind].append(time.perf_counter() - t0)
            if kind == "copies":  # the same blobs again: warm
                t0 = time.perf_counter()
                out2 = ck.computeWeightedAverage(blobs, w)
                res[st]["warm"].append(time.perf_counter() - t0)
                del out2
            del out, blobs
apply("base")
print(json.dumps({"what": "bytes-API wavg input GB/s on fresh blobs (first call on them) and warm (second), %d x %d cts, "
                  "%s wire, median of %d alternated rounds" % (Cl, Ka, a.wire, a.rounds),
                  "settings": {st: {k: round(nb / sorted(v)[len(v) // 2] / 1e9, 2) for k, v in d_.items()}
                               for st, d_ in res.items()}}))
