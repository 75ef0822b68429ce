"""Compare the production trace launches of two rocprofv3 kernel traces
(round 6, verdict r05 next #5: the emulated N = 8 sender against N = 1).

For each trace: the trace_simple launches of the production build (no
counting / diagnostic template), in dispatch order; the timed region is the
last `--timed` of them before the verification launches bench.py issues after
timing (bench's plain_kernels_after_timed, read from its JSON line).  Reports
per launch: duration, grid (workgroups), and over the region: the union of
the launch intervals, the mean number of launches in flight (sum of
durations / union), idle gaps, and durations by position in the exchange
batch.

    python tools/trace_compare.py TRACE.csv BENCH.json [TRACE2.csv BENCH2.json ...]
"""
from __future__ import annotations

import csv
import json
import sys

import numpy as np


def load(trace_csv: str, bench_json: str):
    with open(bench_json) as f:
        b = json.loads(f.read().strip().splitlines()[-1])
    rows = [r for r in csv.DictReader(open(trace_csv))
            if r["Kernel_Name"].startswith("void rtamd::(anonymous namespace)::trace_simple<false, false")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    after = int(b["config"].get("plain_kernels_after_timed") or b["roofline"].get("plain_kernels_after_timed") or 0)
    timed = int(b["config"].get("plain_kernels_timed") or b["roofline"].get("plain_kernels_timed") or 0)
    sel = rows[len(rows) - after - timed: len(rows) - after] if timed else rows
    t0 = np.array([int(r["Start_Timestamp"]) for r in sel], np.float64) / 1e6     # ms
    t1 = np.array([int(r["End_Timestamp"]) for r in sel], np.float64) / 1e6
    grid = np.array([int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) // max(1, int(r["Workgroup_Size_X"]))
                     for r in sel])
    return b, t0, t1, grid


def union(t0, t1):
    order = np.argsort(t0)
    tot, cur_s, cur_e = 0.0, None, None
    gaps = []
    for i in order:
        s, e = t0[i], t1[i]
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot, gaps


def main():
    args = sys.argv[1:]
    for tr, bj in zip(args[::2], args[1::2]):
        b, t0, t1, grid = load(tr, bj)
        dur = t1 - t0
        u, gaps = union(t0, t1)
        fr = b["config"].get("frames_per_step", 1) * b["steps"]
        print(f"{tr}: {len(dur)} launches, ms/step {b['ms_per_step']}, union {u:.3f} ms "
              f"({u / b['steps']:.4f} per step), in flight {dur.sum() / u:.2f}, gaps {len(gaps)} "
              f"({sum(gaps):.4f} ms), launch ms mean {dur.mean():.4f} median {np.median(dur):.4f} "
              f"min {dur.min():.4f} max {dur.max():.4f}; grids {sorted(set(grid.tolist()))[:6]}")
        # launch duration per workgroup (a launch's cost per wave tile)
        print(f"   ms per 1000 workgroups: mean {1000 * (dur / grid).mean():.4f}; frames {fr}")


if __name__ == "__main__":
    main()
