"""A/B of packed-arena wavg variants selected by an environment switch (re-read by the library at each switch)
(AB_ENV, default SHELFI_PACK_UNROLL; AB_VARIANTS, comma-separated values) on the BASELINE
shapes, in one process on one box: launches alternate between the variants in rounds, HIP
events around each round, outputs compared bit for bit.  Prints achieved TB/s (the packed
arena's bytes + the uint64 aggregate per launch) per shape and variant, median over rounds.

usage: AB_ENV=SHELFI_PACK_UNROLL AB_VARIANTS=1,2,4 python tools/wavg_packed_ab.py [rounds] [launches]
A variant may set several switches: AB_VARIANTS="SHELFI_PACK_KERNEL=r3,SHELFI_PACK_KERNEL=v4+SHELFI_PACK_UNROLL=8"
(a variant containing '=' names its own VAR=VAL pairs, joined by '+').
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
    ("cfg4big 16x256", 32768, 5, 16, 256),  # cfg4's ring at cfg3's launch size (ramp / tail vs shape)
    ("N8-cts 128x89", 16384, 3, 128, 89),
]
ENV = os.environ.get("AB_ENV", "SHELFI_PACK_UNROLL")
VARIANTS = os.environ.get("AB_VARIANTS", "1,2,4").split(",")
ONLY = os.environ.get("AB_SHAPES")


_SET = set()


def set_variant(v):
    for k in _SET:
        os.environ.pop(k, None)
    _SET.clear()
    if not v:
        m.reload_switches()
        return
    pairs = [p.split("=", 1) for p in v.split("+")] if "=" in v else [(ENV, v)]
    for k, val in pairs:
        os.environ[k] = val
        _SET.add(k)
    m.reload_switches()  # switches are re-read on request only (never on a launch path)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ctxs = {}
    for name, batch, depth, C, K in SHAPES:
        if ONLY and name.split()[0] not in ONLY.split(","):
            continue
        if (batch, depth) not in ctxs:
            ck = m.CKKS("ckks", batch, 52, "", multDepth=depth, seed=7, decodeNoise=False)
            assert ck.genCryptoContextAndKeyGen() == 1
            ctxs[(batch, depth)] = ck
        ck = ctxs[(batch, depth)]
        inf = ck.info()
        L, N = inf["num_towers"], inf["ring_dim"]
        q = inf["moduli"]
        ar = D.Arena(ck, C, K, layout="packed")
        x = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
        for i in range(C):
            for t in range(L):
                x[:, :, t, :].random_(0, q[t])
            ar.put(i, x)
        del x
        out = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
        w = [1.0 / C] * C
        nbytes = ar.buf.numel() * 8 + K * 2 * L * N * 8
        res = {v: [] for v in VARIANTS}
        ref = None
        for r in range(rounds):
            for v in VARIANTS if r % 2 == 0 else VARIANTS[::-1]:
                set_variant(v)
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
            line.append("%s %.4f ms %.3f TB/s (%.3f of 8)" % (v if "=" in v else "%s=%s" % (ENV, v), ms,
                                                               nbytes / ms / 1e9, nbytes / ms / 8e9))
        print(" | ".join(line), flush=True)
        del ar, out, ref
        torch.cuda.empty_cache()
    set_variant("")


if __name__ == "__main__":
    main()
