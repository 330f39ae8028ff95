"""Arena.put(bytes) throughput: one cfg3 learner's upload (714 ciphertexts at 2^15 / L4, 1.5 GB)
as a library blob and as a PALISADE archive, placed into a 2-learner packed arena, with the host
pieces staged through the pinned copy ring (SHELFI_ARENA_STAGER=1) or copied with plain
hipMemcpyAsync from the pageable upload (=0), alternating, median of 3 puts each (the default picks
per upload: one contiguous run -> plain copy, an archive's tower runs -> the ring).
  python tools/arena_put_time.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def main():
    K = 714
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    x = np.random.default_rng(1).uniform(-1, 1, K * 16384)
    blobs = {"blob": ck.encrypt(x)}
    ck.set_wire_format("palisade")
    blobs["archive"] = ck.encrypt(x)
    ck.set_wire_format("shelfi")
    ar = D.Arena(ck, 2, K, layout="packed")
    for name, b in blobs.items():
        res = {"0": [], "1": []}
        for r in range(4):
            for v in ("1", "0") if r % 2 else ("0", "1"):
                os.environ["SHELFI_ARENA_STAGER"] = v
                m.reload_switches()  # re-read on request only (never on a launch path)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ar.put(0, b)
                torch.cuda.synchronize()
                if r:
                    res[v].append(time.perf_counter() - t0)
        line = "%-8s %d bytes" % (name, len(b))
        for v in ("0", "1"):
            t = float(np.median(res[v]))
            line += " | SHELFI_ARENA_STAGER=%s %.1f ms %.1f GB/s" % (v, t * 1e3, len(b) / t / 1e9)
        print(line, flush=True)
    os.environ.pop("SHELFI_ARENA_STAGER", None)


if __name__ == "__main__":
    main()
