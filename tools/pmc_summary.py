#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch of a kernel."""
import collections
import csv
import glob
import sys


def summarise(root, kernel="trace_kernel<false>"):
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{root}/*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


if __name__ == "__main__":
    s = summarise(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "trace_kernel<false>")
    for k, v in sorted(s.items()):
        print(f"{k:32s} {v:16.1f}")
