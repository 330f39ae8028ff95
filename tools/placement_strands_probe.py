#!/usr/bin/env python3
"""Round 6: can the aggregation's block order make the output placement
irrelevant?  Same pairs as tools/placement_probe2.py (arenas A = Arena's own allocation, T = one
allocation [arena | output], H = [output | arena]; outputs: a plain torch.empty buffer, pool views at
4 GiB steps, T's tail, H's head), each timed with wavg_packed's blocks in order and in
SHELFI_WAVG_STRANDS = 16 / 64 / 256 interleaved strands.  Median of alternated rounds.
    python tools/placement_strands_probe.py"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import _lib  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

K, Cn, B, ROUNDS, LAUNCHES = 714, 16, 16384, 3, 3
STRANDS = [int(v) for v in os.environ.get("PROBE_STRANDS", "0,16,64,256").split(",")]
ck = m.CKKS("ckks", B, 52, "", multDepth=3, seed=7, decodeNoise=False)
assert ck.genCryptoContextAndKeyGen() == 1
inf = ck.info()
L, N = inf["num_towers"], inf["ring_dim"]
lib = _lib.load()
x = torch.rand(K * B, device="cuda", dtype=torch.float64) * 2 - 1
ct = D.encrypt(ck, x)
del x
arena = D.Arena(ck, Cn, K, layout="packed")
for i in range(Cn):
    arena.put(i, ct)
del ct
aw = arena.buf.numel()
ow = K * 2 * L * N
wts = (C.c_float * Cn)(*([1.0 / Cn] * Cn))


def launch(bp, op):
    _lib.check(lib.shelfi_dev_wavg_arena(ck._ctx, C.c_void_p(bp), wts, Cn, K, C.c_void_p(op),
                                         C.c_void_p(torch.cuda.current_stream().cuda_stream)), "wavg_arena")


def time_ms(bp, op):
    launch(bp, op)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * LAUNCHES)]
    for i in range(LAUNCHES):
        ev[2 * i].record()
        launch(bp, op)
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    t = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(LAUNCHES))
    return t[len(t) // 2]


T = torch.empty(aw + ow, dtype=torch.int64, device="cuda")
T[:aw].copy_(arena.buf)
plain = torch.empty(ow, dtype=torch.int64, device="cuda")
pool = torch.empty((12 << 30) // 8 + ow, dtype=torch.int64, device="cuda")
H = torch.empty(ow + aw, dtype=torch.int64, device="cuda")
H[ow:].copy_(arena.buf)
torch.cuda.synchronize()
A0, T0, H0 = arena.buf.data_ptr(), T.data_ptr(), H.data_ptr() + ow * 8
outs = {"T.tail": T0 + aw * 8, "H.head": H.data_ptr(), "plain": plain.data_ptr()}
for g in range(0, 13, 4):
    outs["pool+%dG" % g] = pool.data_ptr() + (g << 30)
places = []
for an, ap in (("A", A0), ("T", T0), ("H", H0)):
    for on, op in outs.items():
        places.append(("%s->%s" % (an, on), ap, op))
ref = None
for st in STRANDS:
    os.environ["SHELFI_WAVG_STRANDS"] = str(st)
    m.reload_switches()
    out = torch.empty(ow, dtype=torch.int64, device="cuda")
    launch(A0, out.data_ptr())
    torch.cuda.synchronize()
    if ref is None:
        ref = out.clone()
    assert torch.equal(out, ref), "strand order changed the aggregate"
    del out
    res = {p[0]: [] for p in places}
    for r in range(ROUNDS):
        for lbl, bp, op in (places if r % 2 == 0 else places[::-1]):
            res[lbl].append(time_ms(bp, op))
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    vals = sorted(med.values())
    for k, v in med.items():
        print(json.dumps({"strands": st, "place": k, "ms": round(v, 4)}), flush=True)
    print(json.dumps({"strands": st, "summary": True, "min_ms": round(vals[0], 4), "median_ms": round(vals[len(vals) // 2], 4),
                      "max_ms": round(vals[-1], 4), "plain_vs_min": round(med["A->plain"] / vals[0], 4)}), flush=True)
