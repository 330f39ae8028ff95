#!/usr/bin/env python3
"""Per-ciphertext counters of one EvalMult and one ModReduce (tools/f4_time.py K 0 under
rocprofv3 --pmc): the mult is every dispatch from the first ks_tensor_intt_kernel to the last
ks_finish_blocks (kernel or _ct), the rescale the dispatches after it up to rescale_finish_blocks (kernel or _ct).
usage: f4_counters.py K counter_collection.csv [more.csv ...] -o out.json
Counters summed per phase and divided by K; FETCH_SIZE is doubled (the gfx950 correction of
MI355X_MICROARCH.md) and reported with WRITE_SIZE as HBM bytes."""
import argparse
import collections
import csv
import json


def phases(rows):
    order = sorted({(int(r["Dispatch_Id"]), r["Kernel_Name"]) for r in rows})
    first = next(i for i, (_, k) in enumerate(order) if "ks_tensor_intt_kernel" in k)
    last_m = max(i for i, (_, k) in enumerate(order) if "ks_finish_blocks" in k)
    last_r = max(i for i, (_, k) in enumerate(order) if "rescale_finish_blocks" in k)
    ph = {}
    for i, (d, _) in enumerate(order):
        if first <= i <= last_m:
            ph[d] = "mult"
        elif last_m < i <= last_r:
            ph[d] = "rescale"
    return ph


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("K", type=int)
    ap.add_argument("csv", nargs="+")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    per_kernel = collections.defaultdict(lambda: collections.defaultdict(float))
    for path in a.csv:
        rows = list(csv.DictReader(open(path)))
        ph = phases(rows)
        for r in rows:
            p = ph.get(int(r["Dispatch_Id"]))
            if p is None:
                continue
            name = r["Counter_Name"]
            v = float(r["Counter_Value"])
            tot[p][name] += v
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("shelfi::", "")
            per_kernel[p + ":" + k][name] += v
    res = {"K": a.K}
    for p, c in tot.items():
        d = {n: v / a.K for n, v in c.items()}
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024  # counters are KiB
        res[p] = {n: round(v) for n, v in d.items()}
    res["per_kernel"] = {k: {n: round(v / a.K) for n, v in c.items()} for k, c in sorted(per_kernel.items())}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({p: res[p] for p in ("mult", "rescale") if p in res}))


if __name__ == "__main__":
    main()
