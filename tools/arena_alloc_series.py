#!/usr/bin/env python3
"""wavg (C = 16, K = 714) and a plain torch read over several consecutive 22 GiB
allocations: is the arena's speed a property of the physical memory behind it?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def med(fn, n=8):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[n // 2]


def main():
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    N, L, q = inf["ring_dim"], inf["num_towers"], inf["moduli"]
    C, K = 16, 714
    w = [1.0 / C] * C
    out = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
    out_first = out
    nb = (C + 1) * K * 2 * L * N * 8
    arenas = []
    outs = []
    own_out = os.environ.get("OWN_OUT") == "1"
    for i in range(int(os.environ.get("NA", "6"))):
        if own_out:  # a fresh output buffer allocated right before each arena
            out = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
            outs.append(out)
        ar = D.Arena(ck, C, K, layout="packed")
        v = ar.buf.view(-1, N)
        for t in range(L):
            v[t::L].random_(0, q[t])
        arenas.append(ar)
        tw = med(lambda: ar.wavg(w, out=out))
        tf = med(lambda: ar.wavg(w, out=out_first))
        buf = ar.buf.view(torch.float64)
        tr = med(lambda: torch.sum(buf))
        print("arena %d ptr 0x%x out 0x%x  wavg %.3f ms (%.2f TB/s)  [into the first out %.3f ms]  "
              "torch.sum read %.3f ms (%.2f TB/s)" %
              (i, ar.buf.data_ptr(), out.data_ptr(), tw, nb / tw / 1e9, tf, tr, buf.numel() * 8 / tr / 1e9),
              flush=True)


if __name__ == "__main__":
    main()
