"""How many back-to-back device encrypts (714 ciphertexts, 2^15 / L4) it takes to reach the steady
state, after (a) a memory-bound aggregation loop like bench.py's timed region, (b) an idle second,
(c) the decrypts that precede encrypt in bench.py.  Prints each call's us/ct (HIP events around the
call) so the ramp is visible.
  python tools/enc_warm_probe.py [calls]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    K = 714
    # PREALLOC_GB: HBM taken before the context's scratch is allocated (bench.py's process holds a
    # ~22 GiB arena by the time it times encrypt), to see whether the scratch's placement matters
    pre = float(os.environ.get("PREALLOC_GB", "0"))
    hold = torch.empty(int(pre * (1 << 30)) // 8, dtype=torch.int64, device="cuda") if pre > 0 else None
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    B, L, N, q = inf["batch"], inf["num_towers"], inf["ring_dim"], inf["moduli"]
    x = torch.rand(K * B, device="cuda", dtype=torch.float64) * 2 - 1
    ce = D.encrypt(ck, x)
    # a 16-learner packed arena of K ciphertexts (bench.py's cfg3 shard) for the aggregation loop
    ar = D.Arena(ck, 16, K, layout="packed")
    for i in range(16):
        ar.put(i, ce)
    out = torch.empty_like(ce)
    w = [1.0 / 16] * 16
    dec = D.decrypt(ck, ce, K * B, inf["delta"])
    torch.cuda.synchronize()

    def run_encrypts(tag):
        ts = []
        for _ in range(calls):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            D.encrypt(ck, x, out=ce)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3 / K)
        print("%-22s " % tag + " ".join("%.2f" % t for t in ts), flush=True)

    print("prealloc %.1f GB" % pre, flush=True)
    del hold
    for rep in range(int(os.environ.get("REPS", "2"))):
        for _ in range(200):  # bench.py's timed aggregation loop
            ar.wavg(w, out=out)
        torch.cuda.synchronize()
        run_encrypts("after 200 wavg")
        time.sleep(1.0)
        run_encrypts("after 1 s idle")
        for _ in range(14):  # bench.py's interleaved decrypt timing
            D.decrypt(ck, ce, K * B, inf["delta"], out=dec)
        torch.cuda.synchronize()
        run_encrypts("after 14 decrypts")


if __name__ == "__main__":
    main()
