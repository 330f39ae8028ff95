#!/usr/bin/env python3
"""Per-kernel table of whatever counters an SQ pass collected (sums over dispatches,
then per dispatch), with the wave-cycle fractions where SQ_WAVE_CYCLES is present.
usage: sq_table.py counter_collection.csv"""
import collections
import csv
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(sys.argv[1])):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "probe::").split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        if not k.startswith(("shelfi", "probe")):
            continue
        n = len(disp[k])
        wc = d.get("SQ_WAVE_CYCLES", 0.0)
        parts = ["%s: %d disp" % (k[:60], n)]
        for c, v in sorted(d.items()):
            parts.append("%s=%.4g" % (c.replace("SQ_", ""), v / n))
        if wc:
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                if c in d:
                    parts.append("%s/wave=%.3f" % (c.replace("SQ_", ""), d[c] / wc))
        if d.get("SQ_INSTS_LDS"):
            parts.append("bank_conflict/lds_inst=%.2f" % (d.get("SQ_LDS_BANK_CONFLICT", 0) / d["SQ_INSTS_LDS"]))
        print("\n  ".join(parts))


if __name__ == "__main__":
    main()
