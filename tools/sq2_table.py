#!/usr/bin/env python3
"""Per-kernel table of SQ counter passes (tools/pmc_sq2_encdec.sh): every counter summed over
the kernel's dispatches, the cycle counters also as a fraction of SQ_WAVE_CYCLES (all in
quad-cycles), and instruction counts per dispatch.  usage: sq2_table.py a.csv [b.csv ...]"""
import collections
import csv
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if not k.startswith("shelfi"):
                continue
            c = r["Counter_Name"]
            agg[k][c] += float(r["Counter_Value"])
            disp[k][c].add(r["Dispatch_Id"])
    for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        print(k)
        for c in sorted(d):
            n = max(1, len(disp[k][c]))
            wc = d.get("SQ_WAVE_CYCLES", 0) / max(1, len(disp[k]["SQ_WAVE_CYCLES"]))
            v = d[c] / n
            extra = ("  (%.3f of wave cycles)" % (v / wc)) if wc and ("CYCLES" in c or "ACTIVE" in c or "WAIT" in c) and c != "SQ_WAVE_CYCLES" else ""
            print("  %-24s %14.4g per dispatch%s" % (c, v, extra))


if __name__ == "__main__":
    main()
