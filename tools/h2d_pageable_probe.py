#!/usr/bin/env python3
"""H2D rates straight from pageable Python bytes (the bytes API's input: 16 learner blobs of 64
ciphertexts at 2^15 / L4, ~134 MB each), by slice size, against the same through a pinned bounce
buffer and the library's staged bytes path (computeWeightedAverage, SHELFI_STAGE_TRACE=1 prints its
fill / wait / drain split).  Round 5 probe for the bytes API's 50 GB/s target.
    python tools/h2d_pageable_probe.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import warnings  # noqa: E402

warnings.filterwarnings("ignore")
Cl = 16
blob_bytes = 64 * 2 * 4 * 32768 * 8 + 4096
blobs = [np.random.default_rng(i).integers(0, 255, blob_bytes, dtype=np.uint8).tobytes() for i in range(Cl)]
dev = torch.empty(Cl * blob_bytes, dtype=torch.uint8, device="cuda")
total = Cl * blob_bytes


def run(slice_mib, reps=3):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        off = 0
        for b in blobs:
            src = torch.frombuffer(b, dtype=torch.uint8)
            step = len(b) if slice_mib == 0 else slice_mib << 20
            for s in range(0, len(b), step):
                n = min(step, len(b) - s)
                dev[off + s:off + s + n].copy_(src[s:s + n], non_blocking=True)
            off += len(b)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


# warm
run(0, 1)
for sm in (0, 128, 32, 8, 2):
    dt = run(sm)
    print(json.dumps({"pageable_slices_mib": sm or "whole", "ms": round(dt * 1e3, 2),
                      "GB_per_s": round(total / dt / 1e9, 2)}), flush=True)
# pinned bounce: one 64 MiB pinned buffer pair, CPU copy then DMA (what the staging ring does, single thread)
pin = [torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
torch.cuda.synchronize()
t0 = time.perf_counter()
off = 0
ev = [None, None]
i = 0
for b in blobs:
    src = torch.frombuffer(b, dtype=torch.uint8)
    for s in range(0, len(b), 64 << 20):
        n = min(64 << 20, len(b) - s)
        if ev[i & 1] is not None:
            ev[i & 1].synchronize()
        pin[i & 1][:n].copy_(src[s:s + n])
        dev[off + s:off + s + n].copy_(pin[i & 1][:n], non_blocking=True)
        e = torch.cuda.Event()
        e.record()
        ev[i & 1] = e
        i += 1
    off += len(b)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(json.dumps({"pinned_bounce_1thread_64mib": True, "ms": round(dt * 1e3, 2), "GB_per_s": round(total / dt / 1e9, 2)}),
      flush=True)

# source alignment (round 5): a PALISADE archive's residue range starts after its headers, at any byte
for off in (0, 8, 64, 100, 4096, 4099):
    ts = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o = 0
        for b in blobs:
            src = torch.frombuffer(b, dtype=torch.uint8)
            for s0 in range(off, len(b) - (32 << 20), 32 << 20):
                dev[o:o + (32 << 20)].copy_(src[s0:s0 + (32 << 20)], non_blocking=True)
                o += 32 << 20
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    dt = sorted(ts)[1]
    print(json.dumps({"src_offset": off, "addr_mod_4096": (torch.frombuffer(blobs[0], dtype=torch.uint8).data_ptr() + off) % 4096,
                      "ms": round(dt * 1e3, 2), "GB_per_s": round(o / dt / 1e9, 2)}), flush=True)
