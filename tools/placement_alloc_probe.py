"""Probe: does the way the aggregate buffer is allocated decide the wavg launch's
placement penalty?  One cfg3 arena (16 learners x 714 cts, 2^15 / L4), then output candidates from three
allocators timed against it by the library's own picker (shelfi_dev_wavg_arena_pick_output, 4 launches
each): torch's caching allocator, hipMalloc, and hipExtMallocWithFlags(hipDeviceMallocContiguous).
Prints each candidate's ms, per allocator.

usage: python tools/placement_alloc_probe.py [per_allocator]
"""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import _lib  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

HIP_MALLOC_CONTIGUOUS = 0x4


def main():
    per = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    Cn, K = 16, 714
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    L, N, q = inf["num_towers"], inf["ring_dim"], inf["moduli"]
    ar = D.Arena(ck, Cn, K, layout="packed")
    x = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
    for i in range(Cn):
        for t in range(L):
            x[:, :, t, :].random_(0, q[t])
        ar.put(i, x)
    del x
    torch.cuda.synchronize()
    nbytes = K * 2 * L * N * 8
    # the HIP runtime already in this process (torch's; the library resolves its HIP calls to it)
    hip_path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
    print("HIP runtime:", hip_path, flush=True)
    hip = C.CDLL(hip_path)
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipFree.argtypes = [C.c_void_p]
    cands, kinds, raw = [], [], []
    for _ in range(per):
        t = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
        cands.append(t.data_ptr())
        kinds.append("torch")
        raw.append(t)
    for _ in range(per):
        p = C.c_void_p()
        rc = hip.hipMalloc(C.byref(p), nbytes)
        if rc == 0:
            cands.append(p.value)
            kinds.append("hipMalloc")
            raw.append(p)
        else:
            print("hipMalloc rc", rc, flush=True)
    for _ in range(per):
        p = C.c_void_p()
        rc = hip.hipExtMallocWithFlags(C.byref(p), nbytes, HIP_MALLOC_CONTIGUOUS)
        if rc == 0:
            cands.append(p.value)
            kinds.append("contiguous")
            raw.append(p)
        else:
            print("hipExtMallocWithFlags(contiguous) rc", rc, flush=True)
            break
    w = (C.c_float * Cn)(*([1.0 / Cn] * Cn))
    ptrs = (C.c_void_p * len(cands))(*cands)
    best = C.c_size_t()
    ms = (C.c_float * len(cands))()
    for rep in range(2):
        rc = _lib.load().shelfi_dev_wavg_arena_pick_output(ck._ctx, C.c_void_p(ar.buf.data_ptr()), w, Cn, K, ptrs,
                                                          len(cands), 4, C.byref(best), ms,
                                                          C.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, _lib.load().shelfi_last_error()
        for kind in ("torch", "hipMalloc", "contiguous"):
            v = [round(float(ms[i]), 4) for i in range(len(cands)) if kinds[i] == kind]
            print("rep %d %-10s %s" % (rep, kind, v), flush=True)
        print("rep %d best %d (%s)" % (rep, best.value, kinds[best.value]), flush=True)
    torch.cuda.synchronize()
    for k, r in zip(kinds, raw):
        if k != "torch":
            hip.hipFree(r)


if __name__ == "__main__":
    main()
