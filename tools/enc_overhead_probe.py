#!/usr/bin/env python3
"""Host overhead of one device-resident encrypt / decrypt call: wall time vs HIP events
recorded on the call's stream around it (the difference is time with no kernel of the
call in flight).   K=714 python tools/enc_overhead_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def main():
    K = int(os.environ.get("K", "714"))
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7)
    assert ck.genCryptoContextAndKeyGen() == 1
    B = ck.info()["batch"]
    x = torch.rand(K * B, device="cuda", dtype=torch.float64) * 2 - 1
    out = D.encrypt(ck, x)
    dec = D.decrypt(ck, out, K * B, ck.info()["delta"])
    torch.cuda.synchronize()
    for name, fn in (("encrypt", lambda: D.encrypt(ck, x, out=out)),
                     ("decrypt", lambda: D.decrypt(ck, out, K * B, ck.info()["delta"], out=dec))):
        walls, evs = [], []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e3)
            evs.append(e0.elapsed_time(e1))
        walls.sort()
        evs.sort()
        print("%s K=%d: wall %.3f ms (%.3f us/ct), events %.3f ms (%.3f us/ct)" %
              (name, K, walls[3], walls[3] * 1e3 / K, evs[3], evs[3] * 1e3 / K))
        # where the host time goes: the Python wrapper alone (ctx info + checks)
    t0 = time.perf_counter()
    for _ in range(100):
        ck.info()
    print("ck.info(): %.1f us" % ((time.perf_counter() - t0) * 1e4))


if __name__ == "__main__":
    main()
