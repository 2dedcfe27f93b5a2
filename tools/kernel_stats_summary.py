#!/usr/bin/env python3
"""Condense a rocprofv3 --stats kernel_stats.csv into the table committed under profiles/.

usage: kernel_stats_summary.py <run_kernel_stats.csv> "<command line that produced it>" > out.txt
"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*$", "", name) if not name.startswith("void") else re.sub(r"\((int|float|long|unsigned|rrtmgpnn).*$", "", name)
    return name[:60]


def main():
    path, cmd = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(path)))
    print(cmd)
    print("%-60s %8s %12s %12s %8s" % ("kernel", "calls", "avg_us", "total_ms", "pct"))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        print("%-60s %8d %12.2f %12.3f %8.2f" % (short(r["Name"]), int(r["Calls"]), float(r["AverageNs"]) / 1e3,
                                                float(r["TotalDurationNs"]) / 1e6, float(r["Percentage"])))


if __name__ == "__main__":
    main()
