"""A/B of the bytes API's upload path: computeWeightedAverage of
16 learners x 64 ciphertexts at 2^15/L4 (bench's api_bytes_path sample), alternating
  staged   — pageable upload -> pinned staging ring -> DMA (default), and
  register — each upload page-locked in place for the call (hipHostRegister) and DMA'd
             straight from it (SHELFI_H2D_REGISTER=1, read per call),
in one process; also the library blob vs the PALISADE archive wire format.  Prints ms per
call and input GB/s, median over rounds; outputs must agree.

usage: python tools/h2d_register_ab.py [rounds] [cts_per_learner]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import SHELFI_FHE as m  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    C = 16
    d = os.path.join(ROOT, "gpurun_out", "h2d_keys") + os.sep
    os.makedirs(d, exist_ok=True)
    ck = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    B = ck.info()["batch"]
    for wire in ("shelfi", "palisade"):
        ck.set_wire_format(wire)
        blobs = [ck.encrypt(np.random.default_rng(i).uniform(-1, 1, K * B)) for i in range(C)]
        w = [1.0 / C] * C
        nbytes = sum(len(b) for b in blobs)
        res = {"0": [], "1": []}
        ref = None
        for r in range(rounds):
            for v in ("0", "1") if r % 2 == 0 else ("1", "0"):
                os.environ["SHELFI_H2D_REGISTER"] = v
                t0 = time.perf_counter()
                out = ck.computeWeightedAverage(blobs, w)
                res[v].append(time.perf_counter() - t0)
                if ref is None:
                    ref = out
                else:
                    assert out == ref, "paths disagree"
                del out
        line = ["%s %d x %d cts (%.2f GB in)" % (wire, C, K, nbytes / 1e9)]
        for v, name in (("0", "staged"), ("1", "register")):
            t = float(np.median(res[v]))
            line.append("%s %.2f ms %.1f GB/s (min %.2f)" % (name, t * 1e3, nbytes / t / 1e9, min(res[v]) * 1e3))
        print(" | ".join(line), flush=True)
        del blobs, ref
    os.environ.pop("SHELFI_H2D_REGISTER", None)


if __name__ == "__main__":
    main()
