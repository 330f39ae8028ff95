#!/usr/bin/env python3
"""HBM placement probe for the aggregation's output: one cfg3 shard arena
(16 learners x 714 ciphertexts, 2^15 / L4, packed), and the [K][2][L][N] aggregate written to
  - 'plain':   a torch.empty buffer allocated after the arena,
  - 'pool+o':  views at offset o of one large pool (steps of `--step` MiB plus a few small offsets),
  - 'tail+p':  the tail of a second arena allocation that also holds the output, p bytes after the
               arena's last word (the by-construction candidate).
Each placement's launch time is the median over alternated rounds (HIP events on torch's stream).
Prints one JSON line per placement and a summary line.
    python tools/placement_probe.py [--k 714] [--pool-gib 14] [--step 256] [--rounds 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import ctypes as C  # noqa: E402

import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import _lib  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=714)
ap.add_argument("--c", type=int, default=16)
ap.add_argument("--pool-gib", type=float, default=14.0)
ap.add_argument("--step", type=int, default=256, help="MiB between pool offsets")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--launches", type=int, default=3)
a = ap.parse_args()
K, Cn, B = a.k, a.c, 16384
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
out_words = K * 2 * L * N
weights = [1.0 / Cn] * Cn
wts = (C.c_float * Cn)(*weights)
torch.cuda.synchronize()
del ct


def launch(base_ptr, out_ptr):
    _lib.check(lib.shelfi_dev_wavg_arena(ck._ctx, C.c_void_p(base_ptr), wts, Cn, K, C.c_void_p(out_ptr),
                                         C.c_void_p(torch.cuda.current_stream().cuda_stream)), "wavg_arena")


def time_ms(base_ptr, out_ptr):
    launch(base_ptr, out_ptr)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.launches)]
    for i in range(a.launches):
        ev[2 * i].record()
        launch(base_ptr, out_ptr)
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    t = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(a.launches))
    return t[len(t) // 2]


places = []  # (label, base_ptr, out_ptr, keepalive)
plain = torch.empty(out_words, dtype=torch.int64, device="cuda")
places.append(("plain", arena.buf.data_ptr(), plain.data_ptr()))
pool_words = int(a.pool_gib * (1 << 30)) // 8
pool = torch.empty(pool_words, dtype=torch.int64, device="cuda")
offs = [0, 4096, 65536, 1 << 20, 2 << 20, 16 << 20, 64 << 20]
o = a.step << 20
while o + out_words * 8 <= pool_words * 8:
    offs.append(o)
    o += a.step << 20
for o in offs:
    places.append(("pool+%d" % o, arena.buf.data_ptr(), pool.data_ptr() + o))
# a second arena allocation holding arena + pad + output: the same packed image copied in
aw = arena.buf.numel()
pads = [0, 4096, 65536, 2 << 20, 256 << 20]
tail = torch.empty(aw + (max(pads) + out_words * 8) // 8, dtype=torch.int64, device="cuda")
tail[:aw].copy_(arena.buf)
for p in pads:
    places.append(("tail+%d" % p, tail.data_ptr(), tail.data_ptr() + aw * 8 + p))
torch.cuda.synchronize()
def fill_ms(out_ptr):
    """write-only rate of the placement: torch fill_ of a [K][2][L][N] view at out_ptr"""
    views = {plain.data_ptr(): plain}
    if pool.data_ptr() <= out_ptr < pool.data_ptr() + pool_words * 8:
        o = (out_ptr - pool.data_ptr()) // 8
        v = pool[o:o + out_words]
    elif tail.data_ptr() <= out_ptr < tail.data_ptr() + tail.numel() * 8:
        o = (out_ptr - tail.data_ptr()) // 8
        v = tail[o:o + out_words]
    else:
        v = views[out_ptr]
    v.fill_(0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.launches):
        v.fill_(0)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.launches


res = {lbl: [] for lbl, _, _ in places}
fills = {lbl: [] for lbl, _, _ in places}
for r in range(a.rounds):
    for lbl, bp, op in (places if r % 2 == 0 else places[::-1]):
        res[lbl].append(time_ms(bp, op))
        fills[lbl].append(fill_ms(op))
med = {lbl: sorted(v)[len(v) // 2] for lbl, v in res.items()}
best = min(med.values())
ptrs = {lbl: (bp, op) for lbl, bp, op in places}
for lbl, v in med.items():
    bp, op = ptrs[lbl]
    fm = sorted(fills[lbl])[len(fills[lbl]) // 2]
    print(json.dumps({"place": lbl, "ms": round(v, 4), "vs_best": round(v / best, 4),
                      "fill_ms": round(fm, 4), "fill_TBps": round(out_words * 8 / fm / 1e9, 2), "arena_va": hex(bp),
                      "out_va": hex(op), "out_minus_arena_gib": round((op - bp) / (1 << 30), 4)}))
print(json.dumps({"summary": True, "best_ms": round(best, 4), "plain_ms": round(med["plain"], 4),
                  "tail0_ms": round(med["tail+0"], 4), "arena_bytes": aw * 8, "out_bytes": out_words * 8,
                  "slow_places": sum(1 for v in med.values() if v > 1.05 * best), "places": len(med)}))
