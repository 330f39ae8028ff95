#!/usr/bin/env python3
"""Pinned host -> device copy bandwidth with 1, 2 and 4 streams (8 MiB pieces, 1 GiB total),
the shape of the bytes API's staged uploads.   python tools/h2d_streams_probe.py"""
import time

import torch


def main():
    piece, total = 8 << 20, 1 << 30
    n = total // piece
    host = [torch.empty(piece, dtype=torch.uint8).pin_memory() for _ in range(16)]
    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    for ns in (1, 2, 4):
        streams = [torch.cuda.Stream() for _ in range(ns)]
        best = 1e9
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(n):
                with torch.cuda.stream(streams[i % ns]):
                    dev[i * piece:(i + 1) * piece].copy_(host[i % 16], non_blocking=True)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        print("H2D %d stream(s): %.1f GB/s" % (ns, total / best / 1e9))
        for ns2 in (1, 2):
            pass
    # D2H for reference
    for ns in (1, 2):
        streams = [torch.cuda.Stream() for _ in range(ns)]
        best = 1e9
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(n):
                with torch.cuda.stream(streams[i % ns]):
                    host[i % 16].copy_(dev[i * piece:(i + 1) * piece], non_blocking=True)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        print("D2H %d stream(s): %.1f GB/s" % (ns, total / best / 1e9))


if __name__ == "__main__":
    main()
