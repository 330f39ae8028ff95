"""Bytes-API aggregation (16 learners x 64 cts, N=2^15, L=4: bench.py's api_bytes_path sample) vs the
pipeline's chunk size (SHELFI_WAVG_CHUNK_MIB, read per call), alternated call by call in one process,
uint64 blobs and the packed wire; results compared bit for bit.
    python tools/api_chunk_probe.py [MiB ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import numpy as np  # noqa: E402

import SHELFI_FHE as m  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [64, 128, 256, 512]
    Cl, Ka = 16, 64
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7)
    assert ck.genCryptoContextAndKeyGen() == 1
    x = np.random.default_rng(1).uniform(-1, 1, Ka * 16384)
    w = [1.0 / Cl] * Cl
    for wire in ("shelfi", "packed"):
        ck.set_wire_format(wire)
        blobs = [ck.encrypt(x) for _ in range(Cl)]
        ref = None
        res = {s: [] for s in sizes}
        for r in range(5):
            for s in (sizes if r % 2 == 0 else sizes[::-1]):
                os.environ["SHELFI_WAVG_CHUNK_MIB"] = str(s)
                m.reload_switches()  # re-read on request only (never on a launch path)
                ck.computeWeightedAverage(blobs, w)  # warm for this size
                t0 = time.perf_counter()
                out = ck.computeWeightedAverage(blobs, w)
                res[s].append(time.perf_counter() - t0)
                if ref is None:
                    ref = out
                else:
                    assert out == ref, "chunk size changed the aggregate"
        in_bytes = sum(len(b) for b in blobs)
        print(wire, " | ".join("%d MiB %.2f ms (%.1f K ct/s, %.1f GB/s in)" % (
            s, 1e3 * np.median(v), Cl * Ka / np.median(v) / 1e3, in_bytes / np.median(v) / 1e9)
            for s, v in res.items()), flush=True)
        del blobs
    ck.set_wire_format("shelfi")


if __name__ == "__main__":
    main()
