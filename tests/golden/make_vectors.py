#!/usr/bin/env python3
"""Writes tests/golden/vectors/ from the oracle (tests/golden_cases.py defines the
cases).  Run from the repo root after `make -C oracle`:

    python tests/golden/make_vectors.py

The oracle is pinned by the reference's committed PALISADE artifacts
(test_oracle_kat.py); these vectors freeze its outputs for one FedAvg round per
parameter set so that the product (test_gpu_golden.py) and any later oracle change
(test_golden.py) are checked against the same committed numbers.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import golden_cases as G  # noqa: E402
import oracle as O  # noqa: E402
import palisade_fixture as P  # noqa: E402


def main():
    out = os.path.join(HERE, "vectors")
    os.makedirs(out, exist_ok=True)
    keys = P.read_keys(os.path.join(HERE, "palisade") + os.sep)
    for name in G.CASES:
        pk, sk, cts, agg, dec, q, psi = G.oracle_round(O, name, keys)
        rec, arrays = G.summarize(name, pk, sk, cts, agg, dec, full=(name == "cfg1"))
        n = G.CASES[name][3]
        rec["max_abs_err_vs_plain_fedavg"] = float(np.abs(dec - G.plain_fedavg(n)).max())
        rec["moduli"] = [int(x) for x in q]
        rec["weights"] = G.weights()
        with open(os.path.join(out, name + ".json"), "w") as f:
            json.dump(rec, f, indent=1)
        if arrays:
            np.savez(os.path.join(out, name + ".npz"), **arrays)
        print(name, rec["agg_sha256"][:16], rec["max_abs_err_vs_plain_fedavg"])


if __name__ == "__main__":
    main()
