#!/usr/bin/env python3
"""Device encrypt + decrypt of one cfg3 learner (K = 714 ciphertexts, 2^15 / L4) a few
times, for rocprofv3 --kernel-trace --stats (per-kernel time of the encrypt and decrypt
chains) and PMC passes.  Prints us/ct of each call type.
  python tools/encdec_prof.py [K] [reps]"""
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
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    batch, depth = int(os.environ.get("BATCH", "16384")), int(os.environ.get("DEPTH", "3"))
    ck = m.CKKS("ckks", batch, 52, "", multDepth=depth, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    B = inf["batch"]
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.rand(K * B, generator=g, device="cuda", dtype=torch.float64) * 2 - 1
    out = D.encrypt(ck, x)
    dec = D.decrypt(ck, out, K * B, inf["delta"])
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("encrypt", lambda: D.encrypt(ck, x, out=out)),
                     ("decrypt", lambda: D.decrypt(ck, out, K * B, inf["delta"], out=dec)),
                     ("decrypt_flooded", lambda: D.decrypt(ck, out, K * B, inf["delta"], out=dec))):
        ck.set_decode_noise(name == "decrypt_flooded")
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        res[name] = sorted(ts)[len(ts) // 2] * 1e6 / K
    err = float((dec - x).abs().max())
    print("N=%d L=%d K=%d  " % (inf["ring_dim"], inf["num_towers"], K) +
          "  ".join("%s %.3f us/ct" % kv for kv in res.items()) + "  max|dec-x| %.2e" % err)


if __name__ == "__main__":
    main()
