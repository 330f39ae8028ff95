#!/usr/bin/env python3
"""Bytes-API aggregation (16 learners x 64 cts, N=2^15, L=4) vs the staging pool's memcpy
thread count (SHELFI_COPY_THREADS, or the upload share SHELFI_H2D_COPY_THREADS with
VAR=SHELFI_H2D_COPY_THREADS; read when a context creates its Stager).
    [VAR=...] python tools/api_threads_probe.py [threads ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import numpy as np  # noqa: E402

import SHELFI_FHE as m  # noqa: E402


def main():
    counts = [int(a) for a in sys.argv[1:]] or [4, 8, 12, 16]
    Cl, Ka = 16, 64
    base = m.CKKS("ckks", 16384, 52, "/tmp/keys_api_probe/", multDepth=3, seed=7)
    os.makedirs("/tmp/keys_api_probe", exist_ok=True)
    assert base.genCryptoContextAndKeyGen() == 1
    x = np.random.default_rng(1).uniform(-1, 1, Ka * 16384)
    blobs = [base.encrypt(x) for _ in range(Cl)]
    w = [1.0 / Cl] * Cl
    Ke = 512
    xe = np.random.default_rng(2).uniform(-1, 1, Ke * 16384)
    for t in counts:
        os.environ[os.environ.get("VAR", "SHELFI_COPY_THREADS")] = str(t)
        ck = m.CKKS("ckks", 16384, 52, "/tmp/keys_api_probe/", multDepth=3)
        ck.loadCryptoParams()
        ck.computeWeightedAverage(blobs, w)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            ck.computeWeightedAverage(blobs, w)
            ts.append(time.perf_counter() - t0)
        dt = sorted(ts)[2]
        te, td = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            blob = ck.encrypt(xe)
            te.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            ck.decrypt(blob, xe.size)
            td.append(time.perf_counter() - t0)
            del blob
        print("threads %2d: wavg %.1f ms, %.1f K client-ct/s, %.1f GB/s input | encrypt %d cts %.1f ms | "
              "decrypt %.1f ms" % (t, dt * 1e3, Cl * Ka / dt / 1e3, Cl * Ka * 2 * 4 * 32768 * 8 / dt / 1e9,
                                   Ke, sorted(te)[1] * 1e3, sorted(td)[1] * 1e3))
        del ck


if __name__ == "__main__":
    main()
