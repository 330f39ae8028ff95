#!/usr/bin/env python3
"""Chunked encrypt / decrypt probe (2^15 / L4, 714 ciphertexts of one cfg3 learner): the same
714 ciphertexts as ceil(714 / Kc) calls of Kc each, us/ct per chunk size.  Small chunks keep
the per-call scratch (pbuf 3 MiB / ct for encrypt, dbuf 1 MiB / ct for decrypt) inside the
256 MB last-level cache instead of round-tripping through HBM.
  python tools/enc_chunk_probe.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    K = 714
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    B = inf["batch"]
    x = torch.rand(K * B, device="cuda", dtype=torch.float64) * 2 - 1
    out = D.encrypt(ck, x)
    dec = D.decrypt(ck, out, K * B, inf["delta"])
    torch.cuda.synchronize()
    for Kc in (714, 357, 179, 90, 45, 24):
        def enc():
            for a in range(0, K, Kc):
                b = min(K, a + Kc)
                D.encrypt(ck, x[a * B:b * B], out=out[a:b])

        def dcr():
            for a in range(0, K, Kc):
                b = min(K, a + Kc)
                D.decrypt(ck, out[a:b], (b - a) * B, inf["delta"], out=dec[a * B:b * B])

        row = []
        for fn in (enc, dcr):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            row.append(sorted(ts)[len(ts) // 2] * 1e6 / K)
        print("Kc=%4d  encrypt %.3f us/ct  decrypt %.3f us/ct" % (Kc, row[0], row[1]), flush=True)
    print("max|dec-x| %.2e" % float((dec - x).abs().max()))


if __name__ == "__main__":
    main()
