#!/usr/bin/env python3
"""Effective clock per dispatch of the encrypt and decrypt chains (MI355X_MICROARCH.md 'DVFS':
GRBM_GUI_ACTIVE / 8 XCDs / wall time), from one rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace run:
counter_collection.csv joined with kernel_trace.csv on the dispatch id.  A call starts at its first
kernel (fft_inv_cols / fft_inv_whole since round 5: encrypt, ntt_inv_blocks_dec: decrypt); a decrypt is
labelled exact or flooded by its FFT pass's FLOOD argument (tools/encdec_traffic.py flood_arg: fft_fwd_blocks_ct
in rounds 3-4, fft_fwd_cols / fft_fwd_whole since round 5) or a flooding kernel of its own.  Prints per call each kernel's us and GHz, then the
medians per label (and writes them as JSON with -o).
  python tools/grbm_clock.py DIR [-o clock.json]"""
import collections
import csv
import glob
import os
import statistics
import json
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from encdec_traffic import flood_arg  # noqa: E402

STARTS = ("fft_inv_cols", "fft_inv_whole", "ntt_inv_blocks_dec")
FLOOD_KERNELS = ("flood_add_kernel", "decode_stats_kernel", "decode_flood_kernel")


def main():
    d = sys.argv[1]
    out = sys.argv[sys.argv.index("-o") + 1] if "-o" in sys.argv else None
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc or not kt:
        sys.exit("no counter_collection.csv / kernel_trace.csv under %s" % d)
    grbm = collections.defaultdict(float)
    for r in csv.DictReader(open(cc[0])):
        if r.get("Counter_Name") == "GRBM_GUI_ACTIVE":
            grbm[r["Dispatch_Id"]] += float(r["Counter_Value"])
    rows = []
    for r in csv.DictReader(open(kt[0])):
        did = r["Dispatch_Id"]
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        ghz = grbm[did] / 8 / (us * 1e3) if did in grbm and us > 0 else float("nan")
        rows.append((int(r["Start_Timestamp"]), r["Kernel_Name"], us, ghz))
    rows.sort()
    short = lambda n: n.replace("void ", "").replace("shelfi::", "").split("(")[0]
    calls, cur = [], []
    for t, name, us, ghz in rows:
        nm = short(name)
        if nm.startswith(STARTS) and cur:
            calls.append(cur)
            cur = []
        cur.append((nm, us, ghz))
    if cur:
        calls.append(cur)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for c in calls:
        names = [n for n, _, _ in c]
        if not names[0].startswith(STARTS):
            continue
        if names[0].startswith(("fft_inv_cols", "fft_inv_whole")):
            label = "encrypt"
        else:
            label = "flooded" if any(n.startswith(FLOOD_KERNELS) or (n.startswith("fft_fwd") and flood_arg(n) == "true")
                                     for n in names) else "exact"
        print("%-8s " % label + "  ".join("%s %.1fus %.2fGHz" % (n.split("<")[0], us, g) for n, us, g in c
                                         if not n.startswith("__amd")))
        for n, us, g in c:
            if n.startswith(("__amd", "at::")):  # runtime copies / the tool's own torch checks
                continue
            # template instances apart (encrypt's two block passes: NORED towers and the 60-bit one)
            per[label][n].append((us, g))
    res = {}
    for label, ks in per.items():
        print("median %s:" % label)
        res[label] = {}
        for n, v in ks.items():
            us, ghz = statistics.median(x for x, _ in v), statistics.median(g for _, g in v)
            print("   %-60s %8.1f us  %.2f GHz  (%d calls)" % (n, us, ghz, len(v)))
            if not n.startswith("__amd"):
                res[label][n] = {"us": round(us, 1), "ghz": round(ghz, 3), "calls": len(v)}
    if out:
        with open(out, "w") as f:
            json.dump({"what": "median per kernel over the calls of each chain: wall us and effective clock "
                               "GRBM_GUI_ACTIVE / 8 / wall", "chains": res}, f, indent=1)


if __name__ == "__main__":
    main()
