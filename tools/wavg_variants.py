#!/usr/bin/env python3
"""Interleaved A/B timing of wavg variants (tools/wavg_variants.hip) on one GPU.
usage: python tools/wavg_variants.py [K] [C]   (builds tools/build/libwv.so first)"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fhe-fed_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

SO = os.path.join(ROOT, "tools", "build", "libwv.so")
os.makedirs(os.path.dirname(SO), exist_ok=True)
if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(os.path.join(ROOT, "tools", "wavg_variants.hip")):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-o", SO, os.path.join(ROOT, "tools", "wavg_variants.hip")], check=True)


class TC(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("q", "one_shoup", "r30", "r30_shoup", "r60", "r60_shoup")]


class Args(C.Structure):
    _fields_ = [("ptrs", C.c_void_p * 16), ("wl", C.c_uint32 * (16 * 16 * 2)), ("out", C.c_void_p),
                ("rows", C.c_uint64), ("C", C.c_uint32), ("L", C.c_uint32), ("logN", C.c_uint32),
                ("pad", C.c_uint32), ("tc", TC * 16)]


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 714
    Cn = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    import oracle as O
    lib = C.CDLL(SO)
    assert lib.wv_sizeof_args() == C.sizeof(Args), (lib.wv_sizeof_args(), C.sizeof(Args))
    N, L = 1 << 15, 4
    q, _ = O.params_generate(N, L, 52, 60)
    q = [int(x) for x in q]
    delta = float(q[-1])
    a = Args()
    a.rows, a.C, a.L, a.logN = K * 2 * L, Cn, L, 15
    for t in range(L):
        a.tc[t].q = q[t]
        a.tc[t].one_shoup = (1 << 64) // q[t]
        for nm, e in (("r30", 30), ("r60", 60)):
            r = (1 << e) % q[t]
            setattr(a.tc[t], nm, r)
            setattr(a.tc[t], nm + "_shoup", (r << 64) // q[t])
    cts = []
    for c in range(Cn):
        x = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
        for t in range(L):
            x[:, :, t].random_(0, q[t])
        cts.append(x)
        a.ptrs[c] = x.data_ptr()
        W = int(float(np.float32(1.0 / Cn)) * delta + 0.5)
        for t in range(L):
            wt = W % q[t]
            a.wl[(c * 16 + t) * 2] = wt & ((1 << 30) - 1)
            a.wl[(c * 16 + t) * 2 + 1] = wt >> 30
    ref = torch.empty_like(cts[0])
    a.out = ref.data_ptr()
    assert lib.wv_launch(0, C.byref(a), 0, None) == 0
    torch.cuda.synchronize()
    run_copy = True
    variants = {0: "product v1 nt", 2: "v2 nt (4 res/thr)", 100: "ceiling nt",
                104: "read-only 1 stream"}
    # interleaved copies of the learners for chunk sizes 512, 1024, 2048
    total = K * 2 * L * N
    packed = {}
    for V in (1, 2, 4):
        buf = torch.empty(Cn * total, dtype=torch.int64, device="cuda")
        for c in range(Cn):
            assert lib.wv_pack(C.c_void_p(cts[c].data_ptr()), C.c_void_p(buf.data_ptr()), c, Cn, 512 * V,
                               C.c_uint64(total)) == 0
        packed[200 + V] = buf
        variants[200 + V] = "interleaved ch=%d" % (512 * V)
    torch.cuda.synchronize()
    base_ptr0 = a.ptrs[0]

    def run(v, cap=2048):
        if v in packed:
            a.ptrs[0] = packed[v].data_ptr()
        r = lib.wv_launch(v, C.byref(a), cap, None)
        a.ptrs[0] = base_ptr0
        return r

    outs = {}
    for v in variants:
        o = torch.empty_like(cts[0])
        a.out = o.data_ptr()
        assert run(v) == 0
        torch.cuda.synchronize()
        if v < 100 or v in packed:
            assert torch.equal(o, ref), variants[v]
        if v in (102, 103):  # copies overwrite odd learners: regenerate is unnecessary for timing
            pass
        outs[v] = o
    times = {v: [] for v in variants}
    caps = {}
    for rnd in range(8):
        for v in variants:
            a.out = outs[v].data_ptr()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(v)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
    nbytes = (Cn + 1) * K * 2 * L * N * 8
    vbytes = {102: Cn * K * 2 * L * N * 8, 103: Cn * K * 2 * L * N * 8, 104: Cn * K * 2 * L * N * 8}
    for v, ts in times.items():
        nb = vbytes.get(v, nbytes)
        ts = sorted(ts)
        print("%-20s median %.3f ms  min %.3f ms  %.2f TB/s (median)" % (variants[v], ts[len(ts) // 2], ts[0],
                                                                      nb / (ts[len(ts) // 2] * 1e-3) / 1e12))
    for v, cl in caps.items():
        for cap in cl:
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                lib.wv_launch(v, C.byref(a), cap, None)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            print("%-20s cap %5d median %.3f ms  %.2f TB/s" % (variants[v], cap, ts[2], nbytes / (ts[2] * 1e-3) / 1e12))


if __name__ == "__main__":
    main()
