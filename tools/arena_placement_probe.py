#!/usr/bin/env python3
"""Does the arena wavg's speed depend on where its 22 GiB land (allocation order,
allocator churn)?  Same kernel, same shape (C = 16, K = 714), several arenas."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def time_arena(ar, w, out, label):
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
    print("%-40s median %.3f ms  min %.3f" % (label, ts[5], ts[0]), flush=True)


def fill(ar, N, L, q):
    v = ar.buf.view(-1, N)
    for t in range(L):
        v[t::L].random_(0, q[t])


def main():
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    N, L, q = inf["ring_dim"], inf["num_towers"], inf["moduli"]
    C, K = 16, 714
    w = [1.0 / C] * C
    out = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
    a1 = D.Arena(ck, C, K, layout="packed")
    fill(a1, N, L, q)
    time_arena(a1, w, out, "arena 1 (first allocation)")
    # churn: many 1.4 GiB tensors allocated and freed
    junk = [torch.empty(K * 2 * L * N, dtype=torch.int64, device="cuda") for _ in range(16)]
    del junk
    torch.cuda.empty_cache()
    a2 = D.Arena(ck, C, K, layout="packed")
    fill(a2, N, L, q)
    time_arena(a2, w, out, "arena 2 (after churn, cache emptied)")
    time_arena(a1, w, out, "arena 1 again")
    junk = [torch.empty(K * 2 * L * N // 7, dtype=torch.int64, device="cuda") for _ in range(60)]
    a3 = D.Arena(ck, C, K, layout="packed")
    fill(a3, N, L, q)
    del junk
    time_arena(a3, w, out, "arena 3 (amid small allocations)")
    print(torch.cuda.memory_allocated() / 2**30, "GiB allocated")


if __name__ == "__main__":
    main()
