#!/usr/bin/env python3
"""Arena wavg at a fixed ~22 GiB of learner data per GPU and growing learner counts
(C = 16 is the learner-sharded cfg3 shard; C = 128, K = 89 is what a rank holds in
the ciphertext-sharded cfg3 layout at 8 GPUs).  Random residues (timing only)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def main():
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    N, L, q = inf["ring_dim"], inf["num_towers"], inf["moduli"]
    for C in [int(x) for x in os.environ.get("CS", "16,32,64,128").split(",")]:
        K = 714 * 16 // C
        ar = D.Arena(ck, C, K, layout="packed")
        v = ar.buf.view(-1, N)  # rows of N residues; towers cycle with the row index
        for t in range(L):
            v[t::L].random_(0, q[t])
        w = [1.0 / C] * C
        out = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
        ar.wavg(w, out=out)
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ar.wavg(w, out=out)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        nb = (C + 1) * K * 2 * L * N * 8
        print("C=%4d K=%4d  median %.3f ms  %.2f TB/s  %.2f M client-ct/s" %
              (C, K, ts[5], nb / (ts[5] * 1e-3) / 1e12, C * K / (ts[5] * 1e-3) / 1e6), flush=True)
        del ar, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
