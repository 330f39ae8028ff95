#!/usr/bin/env python3
"""§8 f4 timing: EvalMult (tensor + HYBRID relinearization) and ModReduce of K ciphertext
pairs at 2^15 / L4 (cfg2/3's ring), HIP events around each call on torch's stream.
    python tools/f4_time.py [K] [reps] [json_out]
Prints one JSON object: per-ciphertext microseconds of mult and rescale (median of reps).
reps = 0: exactly one mult and one rescale after setup, no warm-up (for rocprofv3 --pmc
passes; tools/f4_counters.py attributes the dispatches)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ck = m.CKKS("ckks", int(os.environ.get("BATCH", "16384")), 52, "", multDepth=int(os.environ.get("DEPTH", "3")),
           seed=7, decodeNoise=False)
assert ck.genCryptoContextAndKeyGen() == 1
ck.evalMultKeyGen()
inf = ck.info()
S = inf["batch"]
a = D.encrypt(ck, torch.rand(K * S, device="cuda", dtype=torch.float64) * 2 - 1)
b = D.encrypt(ck, torch.rand(K * S, device="cuda", dtype=torch.float64) * 2 - 1)
out = torch.empty_like(a)
r = torch.empty((K, 2, inf["num_towers"] - 1, inf["ring_dim"]), dtype=a.dtype, device=a.device)
D.mult(ck, a, b, out=out)  # warm-up: tables, scratch (or the one profiled call)
D.rescale(ck, out, out=r)
torch.cuda.synchronize()
if reps == 0:
    print(json.dumps({"K": K, "profiled": "one mult + one rescale"}))
    sys.exit(0)


def timed(fn):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


t_mult = timed(lambda: D.mult(ck, a, b, out=out))
t_res = timed(lambda: D.rescale(ck, out, out=r))
ek = ck.eval_key_info()
res = {"K": K, "ring_dim": inf["ring_dim"], "towers": inf["num_towers"], "dnum": ek["dnum"],
       "special_primes": len(ek["special_moduli"]), "mult_ms": round(t_mult, 4),
       "mult_us_per_ct": round(1e3 * t_mult / K, 3), "rescale_ms": round(t_res, 4),
       "rescale_us_per_ct": round(1e3 * t_res / K, 3)}
print(json.dumps(res))
if len(sys.argv) > 3:
    with open(sys.argv[3], "w") as f:
        json.dump(res, f, indent=1)
