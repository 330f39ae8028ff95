#!/usr/bin/env python3
"""Concise per-kernel summary of a rocprofv3 *_kernel_stats.csv: calls, average and
total microseconds, sorted by total.  usage: kstat_summary.py stats.csv [name-width]"""
import csv
import sys


def main():
    path = sys.argv[1]
    width = int(sys.argv[2]) if len(sys.argv) > 2 else 70
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows:
        print("%-*s calls=%5s avg_us=%10.2f total_ms=%9.3f" % (width, r["Name"][:width], r["Calls"],
                                                               float(r["AverageNs"]) / 1e3,
                                                               float(r["TotalDurationNs"]) / 1e6))


if __name__ == "__main__":
    main()
