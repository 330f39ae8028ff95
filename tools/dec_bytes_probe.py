#!/usr/bin/env python3
"""decrypt(bytes) through the staging pipeline (2^15 / L4): K ciphertexts encrypted to a blob, then
`ck.decrypt(blob, n)` timed (median of reps), exact and flooded decode, library blob and PALISADE
archive.  Set SHELFI_STAGE_TRACE=1 for the per-slot trace of the last call.
  python tools/dec_bytes_probe.py [K] [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import SHELFI_FHE as m  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    B = ck.info()["batch"]
    x = np.random.default_rng(1).uniform(-1, 1, K * B)
    for wire in ("shelfi", "palisade"):
        ck.set_wire_format(wire)
        blob = ck.encrypt(x)
        for flood in (False, True):
            ck.set_decode_noise(flood)
            out = ck.decrypt(blob, K * B)
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                out = ck.decrypt(blob, K * B)
                ts.append(time.perf_counter() - t0)
            ms = sorted(ts)[reps // 2] * 1e3
            print("%-8s flood=%d K=%d blob %.1f MB: %.2f ms (%.1f K ct/s, %.1f GB/s of blob), max|dec-x| %.1e"
                  % (wire, flood, K, len(blob) / 1e6, ms, K / ms, len(blob) / ms / 1e6,
                     float(np.abs(out - x).max())), flush=True)


if __name__ == "__main__":
    main()
