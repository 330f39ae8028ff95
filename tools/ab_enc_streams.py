#!/usr/bin/env python3
"""Round 6 probe: the device encrypt of one learner in n chunks over two streams (SHELFI_ENC_STREAMS=n) against
one chunk, in one process, alternated; the ciphertexts compared bit for bit (same seed).
Measured 2026-10-18 and removed (profiles/r06f/enc_streams_ab.txt): cfg4 K = 32 9.29 -> 10.2 / 12.2 us/ct with
2 / 4 chunks, K = 256 8.3 -> 8.5 / 8.6, cfg3 K = 64 3.21 -> 3.56 / 4.9, K = 714 2.50 -> 2.46 / 2.52 (the switch
no longer exists; the script needs the probe build).
    BATCH=32768 DEPTH=5 python tools/ab_enc_streams.py K [reps] [variants, default 1,2,4]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    variants = (sys.argv[3] if len(sys.argv) > 3 else "1,2,4").split(",")
    batch, depth = int(os.environ.get("BATCH", "16384")), int(os.environ.get("DEPTH", "3"))
    ck = m.CKKS("ckks", batch, 52, "", multDepth=depth, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.rand(K * inf["batch"], generator=g, device="cuda", dtype=torch.float64) * 2 - 1
    out = D.encrypt(ck, x)
    ref = None
    times = {v: [] for v in variants}
    for r in range(5):
        for v in (variants if r % 2 == 0 else variants[::-1]):
            os.environ["SHELFI_ENC_STREAMS"] = v
            m.reload_switches()
            ck.set_seed(11)
            D.encrypt(ck, x, out=out)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref), "variant %s changed the ciphertexts" % v
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                D.encrypt(ck, x, out=out)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            times[v].append(sorted(ts)[len(ts) // 2] * 1e6 / K)
    os.environ.pop("SHELFI_ENC_STREAMS", None)
    m.reload_switches()
    print("N=%d L=%d K=%d  " % (inf["ring_dim"], inf["num_towers"], K) +
          "  ".join("streams=%s %s us/ct" % (v, "/".join("%.2f" % t for t in times[v])) for v in variants) +
          "  (bit-identical)")


if __name__ == "__main__":
    main()
