#!/usr/bin/env python3
"""HBM bytes per wavg launch from rocprofv3 PMC passes (separate FETCH_SIZE and
WRITE_SIZE runs, as MI355X_MICROARCH.md §HBM prescribes):

  bytes = 2 * FETCH_SIZE * 1024   (gfx950 FETCH_SIZE reports half of a 16-B/lane
                                   coalesced streaming read; unit KiB)
        +     WRITE_SIZE * 1024   (exact for 16-B/lane streaming stores)

usage: pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv
           --kernel wavg_kernel --workload cfg3 --learners 16 -o profiles/wavg_traffic.json
"""
import argparse
import csv
import json
import statistics


def per_dispatch(path, counter, kernel):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel not in row.get("Kernel_Name", ""):
                continue
            if row.get("Counter_Name") != counter:
                continue
            d = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--kernel", default="wavg_kernel")
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--learners", type=int, default=16)
    ap.add_argument("--algorithmic-bytes", type=float, default=None)
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    f = per_dispatch(a.fetch_csv, "FETCH_SIZE", a.kernel)
    w = per_dispatch(a.write_csv, "WRITE_SIZE", a.kernel)
    if not f or not w:
        raise SystemExit("no %s dispatches with FETCH_SIZE/WRITE_SIZE found" % a.kernel)
    fetch_kb, write_kb = statistics.median(f), statistics.median(w)
    hbm = 2.0 * fetch_kb * 1024 + write_kb * 1024
    out = {"kernel": a.kernel, "workload": a.workload, "learners": a.learners,
           "dispatches": [len(f), len(w)], "fetch_size_kb_median": fetch_kb,
           "write_size_kb_median": write_kb, "hbm_bytes_per_launch": hbm,
           "correction": "2*FETCH_SIZE (gfx950 half-count on 16B/lane streaming reads) + WRITE_SIZE, KiB->B"}
    if a.algorithmic_bytes:
        out["algorithmic_bytes_per_launch"] = a.algorithmic_bytes
        out["traffic_over_algorithmic"] = hbm / a.algorithmic_bytes
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
