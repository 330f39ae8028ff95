#!/usr/bin/env python3
"""Counterpart of the reference's code/benchmark.py (and benchmark_selection*.py):
N simulated clients of a synthetic model, encrypted FedAvg through SHELFI_FHE, the
same printed timing lines (benchmark.py:539-543).

  python tools/fedavg_benchmark.py --model resnet18 --clients 3            # benchmark.py
  python tools/fedavg_benchmark.py --model resnet50 --select rate --rate 0.1  # selection_rate
  python tools/fedavg_benchmark.py --model resnet18 --pack                 # one vector per client
  python tools/fedavg_benchmark.py --model resnet50 --select mask --rate 0.1 --pack  # masking.py top-k
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))

import numpy as np  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import fedavg as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=["lenet5", "resnet18", "resnet50"], default="resnet18")
    ap.add_argument("--clients", type=int, default=3)          # benchmark.py:420
    ap.add_argument("--batch", type=int, default=4096)         # benchmark.py:477
    ap.add_argument("--scale-bits", type=int, default=52)
    ap.add_argument("--mult-depth", type=int, default=1)
    ap.add_argument("--cryptodir", default=os.path.join(ROOT, "tests", "golden", "palisade") + "/")
    ap.add_argument("--select", choices=["all", "layers", "rate", "mask"], default="all")
    ap.add_argument("--rate", type=float, default=0.1,
                    help="rate: encrypted prefix fraction; mask: top-k fraction of each key")
    ap.add_argument("--layers", default="")
    ap.add_argument("--pack", action="store_true")
    ap.add_argument("--wire", choices=["shelfi", "palisade", "packed"], default="shelfi",
                    help="bytes format of the ciphertexts (palisade = the reference's own archives, "
                         "packed = this library's blob at the moduli's bit widths)")
    a = ap.parse_args()
    shapes = {"lenet5": F.lenet5_shapes(), "resnet18": F.resnet_shapes(18),
              "resnet50": F.resnet_shapes(50)}[a.model]
    print(sum(int(np.prod(s)) for s in shapes.values()))  # benchmark.py:426
    states = F.synthetic_states(shapes, a.clients)
    t0 = time.time()
    ck = m.CKKS("ckks", a.batch, a.scale_bits, a.cryptodir, multDepth=a.mult_depth)
    if a.mult_depth == 1 and a.batch == 4096:
        ck.loadCryptoParams()  # benchmark.py:481 (the reference's own keys)
    else:
        ck.genCryptoContextAndKeyGen()
    if a.wire != "shelfi":
        ck.set_wire_format(a.wire)
    t_init = time.time() - t0
    masks = None
    if a.select == "mask":  # masking.py:15-21 top-k of a sensitivity map (synthetic: |grad| ~ U(0,1))
        rs = np.random.default_rng(11)
        masks = {k: F.top_k_mask(rs.random(v.size), a.rate) for k, v in states[0].items()}
    sel = F.Selection(a.select, rate=a.rate, layers=[int(x) for x in a.layers.split(",") if x], masks=masks)
    run = F.SecureFedAvg(ck, sel, pack=a.pack)
    agg, t = run.run(states)
    print("Init Time: {}".format(t_init))
    print(run.report())
    exp = {k: sum(s[k] for s in states) * float(np.float32(1 / a.clients)) for k in states[0]}
    err = max(float(np.abs(agg[k] - exp[k]).max()) for k in exp)
    print("max |FHE - plain FedAvg| = %.3g" % err)


if __name__ == "__main__":
    main()
