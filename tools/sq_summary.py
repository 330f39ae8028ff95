#!/usr/bin/env python3
"""Per-kernel summary of an SQ counter pass (tools/pmc_sq.sh): fraction of wave cycles
issuing VALU / any instruction, parked (s_waitcnt / barrier: SQ_WAIT_ANY) and
issue-stalled (SQ_WAIT_INST_ANY), plus instruction counts, summed over dispatches.
usage: sq_summary.py sq_counter_collection.csv > profiles/r01_sq_counters.md"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    vgpr = {}
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
        vgpr[k] = r["VGPR_Count"]
    print("| kernel | dispatches | VALU issue | any issue | parked (waitcnt/barrier) | issue-stalled | VALU insts | LDS insts |")
    print("|---|---|---|---|---|---|---|---|")
    for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = d.get("SQ_WAVE_CYCLES", 0)
        if not wc or not k.startswith("shelfi"):
            continue
        print("| `%s` | %d | %.2f | %.2f | %.2f | %.2f | %.3g | %.3g |" % (
            k, len(disp[k]), d["SQ_ACTIVE_INST_VALU"] / wc, d["SQ_ACTIVE_INST_ANY"] / wc,
            d["SQ_WAIT_ANY"] / wc, d["SQ_WAIT_INST_ANY"] / wc, d["SQ_INSTS_VALU"], d["SQ_INSTS_LDS"]))


if __name__ == "__main__":
    main()
