#!/usr/bin/env python3
"""Bytes-API aggregation (computeWeightedAverage of 16 learners x 64 cts at 2^15 / L4: what
benchmark.py:506-518 times) per wire format and upload setting (round 5: direct pageable uploads by
default, SHELFI_H2D_DIRECT=0 the pinned staging ring; SHELFI_WAVG_CHUNK_MIB), plus the raw H2D rates on
this box (pinned and pageable, torch) and its NUMA layout.  Each setting gets a fresh context (switches
are read when it is created); SHELFI_STAGE_TRACE=1 makes the library print fill / wait / drain times to
stderr.  Prints JSON lines.
    python tools/bytes_api_probe.py"""
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import numpy as np  # noqa: E402


def topology():
    t = {"affinity_cpus": len(os.sched_getaffinity(0))}
    try:
        t["lscpu_numa"] = [l.strip() for l in subprocess.run(["lscpu"], capture_output=True, text=True).stdout.splitlines()
                           if "NUMA" in l]
    except OSError:
        pass
    nodes = {}
    for f in glob.glob("/sys/class/drm/card*/device/numa_node"):
        try:
            nodes[f.split("/")[4]] = open(f).read().strip()
        except OSError:
            pass
    t["drm_numa_node"] = nodes
    return t


def raw_h2d():
    import torch

    n = 512 << 20
    out = {}
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    for name, host in (("pinned", torch.empty(n, dtype=torch.uint8, pin_memory=True)),
                       ("pageable", torch.empty(n, dtype=torch.uint8))):
        host.fill_(1)
        dev.copy_(host, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(4):
            dev.copy_(host, non_blocking=True)
        torch.cuda.synchronize()
        out[name + "_GBps"] = round(4 * n / (time.perf_counter() - t0) / 1e9, 1)
    return out


def main():
    print(json.dumps({"topology": topology()}), flush=True)
    print(json.dumps({"raw_h2d_512MiB": raw_h2d()}), flush=True)
    import SHELFI_FHE as m

    Cl, Ka, B = 16, 64, 16384
    d = "/tmp/keys_bytes_probe/"
    os.makedirs(d, exist_ok=True)
    base = m.CKKS("ckks", B, 52, d, multDepth=3, seed=7)
    assert base.genCryptoContextAndKeyGen() == 1
    x = np.random.default_rng(1).uniform(-1, 1, Ka * B)
    inputs = {}
    for fmt in ("palisade", "shelfi", "packed"):
        base.set_wire_format(fmt)
        inputs[fmt] = [base.encrypt(x) for _ in range(Cl)]
    w = [1.0 / Cl] * Cl
    settings = [("default", {}), ("ring", {"SHELFI_H2D_DIRECT": "0"}),
                ("direct_chunk256", {"SHELFI_WAVG_CHUNK_MIB": "256"}),
                ("direct_chunk1024", {"SHELFI_WAVG_CHUNK_MIB": "1024"})]
    for name, env in settings:
        for k in ("SHELFI_COPY_THREADS", "SHELFI_H2D_COPY_THREADS", "SHELFI_H2D_DIRECT", "SHELFI_WAVG_CHUNK_MIB"):
            os.environ.pop(k, None)
        os.environ.update(env)
        ck = m.CKKS("ckks", B, 52, d, multDepth=3)
        ck.loadCryptoParams()
        for fmt in ("palisade", "shelfi", "packed") if name in ("default", "ring") else ("palisade",):
            blobs = inputs[fmt]
            nb = sum(len(b) for b in blobs)
            ck.computeWeightedAverage(blobs, w)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                ck.computeWeightedAverage(blobs, w)
                ts.append(time.perf_counter() - t0)
            dt = sorted(ts)[2]
            print(json.dumps({"setting": name, "wire": fmt, "ms": round(dt * 1e3, 2),
                              "client_ct_per_s": round(Cl * Ka / dt, 1), "input_GB_per_s": round(nb / dt / 1e9, 2)}),
                  flush=True)
        del ck


if __name__ == "__main__":
    main()
