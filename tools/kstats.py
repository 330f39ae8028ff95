"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv (name, calls, avg us, %).
  python tools/kstats.py gpurun_out/prof/p_kernel_stats.csv [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print("%-64s %5s %11.1f %7s" % (r["Name"][:64], r["Calls"], float(r["AverageNs"]) / 1000,
                                    r["Percentage"]))
