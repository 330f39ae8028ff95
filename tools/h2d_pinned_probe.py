#!/usr/bin/env python3
"""H2D rate from PINNED host memory by copy size (round 5: the bytes API's staging ring DMAs 8 MiB pinned
slots and its uploads ran ~47 GB/s while warm pageable copies of 32 MiB ran 53-55).  A warm 2 GiB pinned
buffer is copied to the device in slices of 2..128 MiB, on one stream and alternated over two; run it under
`rocprofv3 --kernel-trace --stats` to see whether the copies run as blit kernels or on the DMA engines.
    python tools/h2d_pinned_probe.py"""
import json
import time

import torch

total = 2 << 30
src = torch.empty(total, dtype=torch.uint8, pin_memory=True)
src.fill_(7)
dev = torch.empty(total, dtype=torch.uint8, device="cuda")
streams = [torch.cuda.Stream(), torch.cuda.Stream()]


def run(slice_mib, nstreams, reps=3):
    ts = []
    step = slice_mib << 20
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, s in enumerate(range(0, total, step)):
            with torch.cuda.stream(streams[i % nstreams]):
                dev[s:s + step].copy_(src[s:s + step], non_blocking=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


run(32, 1, 1)
for ns in (1, 2):
    for sm in (2, 4, 8, 16, 32, 64, 128):
        dt = run(sm, ns)
        print(json.dumps({"pinned_slice_mib": sm, "streams": ns, "ms": round(dt * 1e3, 2),
                          "GB_per_s": round(total / dt / 1e9, 2)}), flush=True)
