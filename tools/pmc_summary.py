#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch of a kernel."""
import collections
import csv
import glob
import sys


def bench_rows(rows):
    """The dispatches of the bench's own launches: grids above 2/3 of the
    largest.  A launch of F frames has about F x the grid of a one-frame
    launch, so with bench.py --batch F > 1 (the N = 1 default is 2) this
    drops the one-frame verification launches after the timed region
    (rt_render_tile_device); with F = 1 every grid is about one frame's
    (learned orders vary it by a few wave tiles) and all are kept."""
    if not rows:
        return rows
    g = max(int(r["Grid_Size"]) for r in rows)
    return [r for r in rows if 3 * int(r["Grid_Size"]) > 2 * g]


def summarise(root, kernel="trace_kernel<false>"):
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{root}/*/run_counter_collection.csv")):
        for r in bench_rows([r for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"]]):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


if __name__ == "__main__":
    s = summarise(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "trace_kernel<false>")
    for k, v in sorted(s.items()):
        print(f"{k:32s} {v:16.1f}")
