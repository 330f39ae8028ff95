#!/usr/bin/env python3
"""Bytes-API aggregation (computeWeightedAverage, 16 learners x 64 cts at 2^15 / L4) per upload setting,
alternated round by round in ONE process and one context (settings are switch sets re-read with
SHELFI_FHE.reload_switches), so box state drifts hit every setting alike; outputs checked byte-identical.
--numa local|remote|none first binds this process (and the threads it starts later) to the CPUs of the
GPU's NUMA node (or the other node) and allocates the learners' blobs there.
    python tools/bytes_api_ab.py [--numa local] [--rounds 5] base SHELFI_H2D_DIRECT=0 ..."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import numpy as np  # noqa: E402


def gpu_numa_node(dev=0):
    """NUMA node of HIP device `dev` (its PCI bus id -> /sys/bus/pci/devices/.../numa_node), or -1."""
    try:
        try:
            hip = ctypes.CDLL("libamdhip64.so")
        except OSError:
            hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, dev) != 0:
            return -1
        return int(open("/sys/bus/pci/devices/%s/numa_node" % buf.value.decode().lower()).read())
    except OSError:
        return -1


def node_cpus(node):
    out = set()
    for part in open("/sys/devices/system/node/node%d/cpulist" % node).read().strip().split(","):
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


ap = argparse.ArgumentParser()
ap.add_argument("--numa", choices=["none", "local", "remote"], default="none")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--wire", default="palisade")
ap.add_argument("settings", nargs="+")
a = ap.parse_args()
info = {"numa": a.numa, "gpu_node": gpu_numa_node()}
if a.numa != "none" and info["gpu_node"] >= 0:
    nodes = sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node") and d[4:].isdigit())
    want = info["gpu_node"] if a.numa == "local" else next((n for n in nodes if n != info["gpu_node"]), info["gpu_node"])
    cpus = node_cpus(want) & os.sched_getaffinity(0)
    if cpus:
        os.sched_setaffinity(0, cpus)
        info["bound_node"], info["cpus"] = want, len(cpus)
import SHELFI_FHE as m  # noqa: E402

Cl, Ka, B = 16, 64, 16384
d = "/tmp/keys_bytes_ab/"
os.makedirs(d, exist_ok=True)
ck = m.CKKS("ckks", B, 52, d, multDepth=3, seed=7)
assert ck.genCryptoContextAndKeyGen() == 1
ck.set_wire_format(a.wire)
x = np.random.default_rng(1).uniform(-1, 1, Ka * B)
blobs = [ck.encrypt(x) for _ in range(Cl)]
nb = sum(len(b) for b in blobs)
w = [1.0 / Cl] * Cl
keys = sorted({kv.split("=")[0] for st in a.settings if st != "base" for kv in st.split(",")})


def apply(st):
    for k in keys:
        os.environ.pop(k, None)
    if st != "base":
        for kv in st.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
    m.reload_switches()


ref = ck.computeWeightedAverage(blobs, w)
res = {st: [] for st in a.settings}
for r in range(a.rounds):
    for st in (a.settings if r % 2 == 0 else a.settings[::-1]):
        apply(st)
        out = ck.computeWeightedAverage(blobs, w)  # warm this setting's buffers
        assert out == ref, st
        kept = []  # results freed after the clock stops (benchmark.py keeps each aggregate)
        t0 = time.perf_counter()
        for _ in range(3):
            kept.append(ck.computeWeightedAverage(blobs, w))
        res[st].append((time.perf_counter() - t0) / 3)
        del kept
apply("base")
print(json.dumps({"what": "bytes-API wavg, %d learners x %d cts, %s wire, %.1f MB in; median of %d alternated rounds x 3 calls"
                  % (Cl, Ka, a.wire, nb / 1e6, a.rounds), **info,
                  "settings": {st: {"ms": round(sorted(v)[len(v) // 2] * 1e3, 2),
                                    "input_GB_per_s": round(nb / sorted(v)[len(v) // 2] / 1e9, 2)}
                               for st, v in res.items()}}))
