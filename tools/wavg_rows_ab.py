"""(Round-3 probe of the uint64 arena kernel, before the packed arena: since then the arena runs
wavg_packed, which ignores SHELFI_WAVG_ROWS; tools/wavg_packed_ab.py is its A/B tool.)
A/B of the arena wavg kernel's rows per block (SHELFI_WAVG_ROWS=1|2, read per launch) on
the BASELINE shapes, in one process on one box: launches alternate between the variants in
rounds, HIP events around each round.  Prints achieved TB/s (algorithmic bytes
(C+1) K 2 L N 8 per launch) per shape and variant, median over rounds.

usage: python tools/wavg_rows_ab.py [rounds] [launches_per_round]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

SHAPES = [  # name, batch, multDepth, C, K
    ("cfg2 16x4", 16384, 3, 16, 4),
    ("cfg5 8x156", 16384, 3, 8, 156),
    ("cfg3 16x714", 16384, 3, 16, 714),
    ("cfg4 16x32", 32768, 5, 16, 32),
    ("C2 2x714", 16384, 3, 2, 714),
    ("C4 4x714", 16384, 3, 4, 714),
    ("C8 8x714", 16384, 3, 8, 714),
    ("C12 12x476", 16384, 3, 12, 476),
]
VARIANTS = os.environ.get("AB_VARIANTS", "1,2,4").split(",")


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ctxs = {}
    for name, batch, depth, C, K in SHAPES:
        if (batch, depth) not in ctxs:
            ck = m.CKKS("ckks", batch, 52, "", multDepth=depth, seed=7, decodeNoise=False)
            assert ck.genCryptoContextAndKeyGen() == 1
            ctxs[(batch, depth)] = ck
        ck = ctxs[(batch, depth)]
        inf = ck.info()
        L, N = inf["num_towers"], inf["ring_dim"]
        q = inf["moduli"]
        ar = D.Arena(ck, C, K, layout="packed")
        for i in range(C):
            x = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
            for t in range(L):
                x[:, :, t, :].random_(0, q[t])
            ar.put(i, x)
            del x
        out = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
        w = [1.0 / C] * C
        nbytes = (C + 1) * K * 2 * L * N * 8
        res = {v: [] for v in VARIANTS}
        ref = None
        for r in range(rounds):
            for v in VARIANTS if r % 2 == 0 else VARIANTS[::-1]:
                os.environ["SHELFI_WAVG_ROWS"] = v
                m.reload_switches()  # re-read on request only (never on a launch path)
                ar.wavg(w, out=out)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(per):
                    ar.wavg(w, out=out)
                b.record()
                torch.cuda.synchronize()
                res[v].append(a.elapsed_time(b) / per)
                if ref is None:
                    ref = out.clone()
                else:
                    assert torch.equal(out, ref), "variants disagree"
        line = [name]
        for v in VARIANTS:
            ms = float(np.median(res[v]))
            line.append("R=%s %.4f ms %.3f TB/s (%.3f of 8)" % (v, ms, nbytes / ms / 1e9, nbytes / ms / 8e9))
        print(" | ".join(line), flush=True)
        del ar, out, ref
        torch.cuda.empty_cache()
    os.environ.pop("SHELFI_WAVG_ROWS", None)


if __name__ == "__main__":
    main()
