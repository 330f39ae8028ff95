#!/usr/bin/env python3
"""Arena wavg speed vs the arena's start address: one over-allocated buffer, the
arena placed at different offsets inside it (same physical pages, different virtual
alignment), plus the alignment of fresh allocations."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import _lib  # noqa: E402


def tz(p):
    return (p & -p).bit_length() - 1


def main():
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    N, L, q = inf["ring_dim"], inf["num_towers"], inf["moduli"]
    Cn, K = 16, 714
    lib = _lib.load()
    words = lib.shelfi_arena_words(ck._ctx, Cn, K)
    w = (C.c_float * Cn)(*([1.0 / Cn] * Cn))
    out = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
    slack = (1 << 30) // 8
    big = torch.empty(words + slack, dtype=torch.int64, device="cuda")
    print("big alloc ptr 0x%x (aligned 2^%d)" % (big.data_ptr(), tz(big.data_ptr())), flush=True)
    v = big.view(-1, N)
    for t in range(L):
        v[t::L].random_(0, q[t])
    stream = torch.cuda.current_stream().cuda_stream

    def run(ptr):
        return lib.shelfi_dev_wavg_arena(ck._ctx, C.c_void_p(ptr), w, Cn, K, C.c_void_p(out.data_ptr()),
                                         C.c_void_p(stream))

    base = big.data_ptr()
    for off in (0, 4096, 65536, 1 << 20, 2 << 20, 4 << 20, 64 << 20, 256 << 20, 512 << 20):
        # keep the start a multiple of 64 B; the arena's data is whatever lies there (timing only)
        p = base + off
        assert run(p) == 0
        torch.cuda.synchronize()
        ts = []
        for _ in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(p)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        print("offset %10d (addr aligned 2^%2d): median %.3f ms" % (off, tz(p), ts[4]), flush=True)
    del big
    for i in range(3):
        t = torch.empty(words, dtype=torch.int64, device="cuda")
        print("fresh alloc %d ptr 0x%x aligned 2^%d" % (i, t.data_ptr(), tz(t.data_ptr())), flush=True)


if __name__ == "__main__":
    main()
