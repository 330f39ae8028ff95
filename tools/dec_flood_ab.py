#!/usr/bin/env python3
"""Exact vs flooded device decrypt of K ciphertexts (2^15 / L4 by default), alternated in one
process (exact, flooded, exact, ... with HIP-event-free host timing around each call + sync), so
both see the same clock / power state: prints the median us/ct of each and of the first half vs
the second half of the rounds (a drift there is the chain slowing under sustained load).
  python tools/dec_flood_ab.py [K] [rounds]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 714
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    batch, depth = int(os.environ.get("BATCH", "16384")), int(os.environ.get("DEPTH", "3"))
    ck = m.CKKS("ckks", batch, 52, "", multDepth=depth, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    B, delta = inf["batch"], inf["delta"]
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.rand(K * B, generator=g, device="cuda", dtype=torch.float64) * 2 - 1
    ct = D.encrypt(ck, x)
    dec = D.decrypt(ck, ct, K * B, delta)
    torch.cuda.synchronize()
    res = {False: [], True: []}
    # ORDER=block: every exact call first, then every flooded one (bench.py's order before round 4)
    block = os.environ.get("ORDER", "alt") == "block"
    seq = ([False] * rounds + [True] * rounds) if block else \
        [f for r in range(rounds) for f in ((False, True) if r % 2 == 0 else (True, False))]
    for flood in seq:
        if True:
            ck.set_decode_noise(flood)
            t0 = time.perf_counter()
            D.decrypt(ck, ct, K * B, delta, out=dec)
            torch.cuda.synchronize()
            res[flood].append((time.perf_counter() - t0) * 1e6 / K)
    err = float((dec - x).abs().max())
    h = rounds // 2
    for flood in (False, True):
        v = res[flood]
        print("%-8s median %.3f us/ct  first half %.3f  second half %.3f  all %s" % (
            "flooded" if flood else "exact", sorted(v)[len(v) // 2], sorted(v[:h])[h // 2],
            sorted(v[h:])[(len(v) - h) // 2], " ".join("%.3f" % t for t in v)))
    print("max|dec - x| %.2e (flooded last)" % err)


if __name__ == "__main__":
    main()
