#!/usr/bin/env python3
"""Device encrypt (and decrypt) time per ciphertext under two settings of a launch-time
switch (the environment variable named by VAR, read by the launch code under test), alternated A/B/A/B in one
process, with the seeded ciphertexts checked bit-identical between the settings.
  VAR=SHELFI_ENC_PARK BATCH=16384 DEPTH=3 K=238 [VALS=0,1] python tools/enc_variant_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def main():
    var = os.environ["VAR"]
    batch, depth = int(os.environ.get("BATCH", "16384")), int(os.environ.get("DEPTH", "3"))
    K = int(os.environ.get("K", "238"))
    flood = os.environ.get("FLOOD", "0") == "1"  # exact decode (comparable across variants) by default
    ck = m.CKKS("ckks", batch, 52, "", multDepth=depth, seed=7, decodeNoise=flood)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    B = inf["batch"]
    g = torch.Generator(device="cuda").manual_seed(3)
    x = (torch.rand(K * B, generator=g, device="cuda", dtype=torch.float64) * 2 - 1)
    vals = os.environ.get("VALS", "0,1").split(",")
    outs, decs = {}, {}
    times = {v: [] for v in vals}
    dtimes = {v: [] for v in vals}
    for rep in range(int(os.environ.get("REPS", "3"))):
        for v in (vals if rep % 2 == 0 else vals[::-1]):
            os.environ[var] = v
            m.reload_switches()  # re-read on request only (never on a launch path)
            ck.set_seed(11)
            out = D.encrypt(ck, x)  # warm (allocations)
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                ck.set_seed(11)
                t0 = time.perf_counter()
                D.encrypt(ck, x, out=out)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            times[v].append(sorted(ts)[2] * 1e3 / K)
            dec = D.decrypt(ck, out, K * B, inf["delta"])
            torch.cuda.synchronize()
            ds = []
            for _ in range(5):
                t0 = time.perf_counter()
                D.decrypt(ck, out, K * B, inf["delta"], out=dec)
                torch.cuda.synchronize()
                ds.append(time.perf_counter() - t0)
            dtimes[v].append(sorted(ds)[2] * 1e3 / K)
            outs[v] = out.clone()
            decs[v] = dec.clone()
    same = all(torch.equal(outs[vals[0]], outs[v]) for v in vals)
    same_dec = flood or all(torch.equal(decs[vals[0]], decs[v]) for v in vals)
    err = float((dec - x).abs().max())
    print("%s N=%d L=%d K=%d identical=%s decrypt_identical=%s max|dec-x|=%.2e" % (
        var, inf["ring_dim"], inf["num_towers"], K, same, same_dec, err))
    for v in vals:
        print("  %s=%-4s encrypt ms/ct %s   decrypt ms/ct %s" % (
            var, v, " ".join("%.5f" % t for t in times[v]), " ".join("%.5f" % t for t in dtimes[v])),
              flush=True)


if __name__ == "__main__":
    main()
