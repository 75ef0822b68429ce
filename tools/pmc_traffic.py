#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from tools/pmc.sh passes.

Usage: python tools/pmc_traffic.py gpurun_out/<TAG> "<kernel substring>[|<kernel substring>...]"
           [--config NAME] [--out FILE] [--merge profiles/pmc_latest.json]

--merge adds (or replaces) the config's record in a multi-config file
{"configs": {NAME: {...}}}, which bench.py reads for its roofline
(SQ_INSTS_VMEM_RD and HBM bytes per launch).

FETCH_SIZE (pass C) is in KiB and, on gfx950, counts 64-B halves of 128-B
requests, so bytes = FETCH_SIZE x 1024 x 2 (MI355X_MICROARCH.md, HBM /
rocprofv3 section).  Hit rates and SQ fractions come from passes A, B and D.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarise  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("kernel")
    ap.add_argument("--config", default="cfg3_50k_1920x1080_b4")
    ap.add_argument("--out", default="")
    ap.add_argument("--source", default="")
    ap.add_argument("--merge", default="", help="multi-config JSON to add this config's record to")
    args = ap.parse_args()
    # A frame may be several launches (heavy tiles + the other tiles): the
    # kernel argument is a "|"-separated list, and per-launch means are summed.
    s = {}
    for name in args.kernel.split("|"):
        for k, v in summarise(args.root, name).items():
            s[k] = s.get(k, 0.0) + v
    if "FETCH_SIZE" not in s:
        sys.exit(f"no FETCH_SIZE rows for kernel {args.kernel!r} under {args.root}")
    out = {
        "kernel": args.kernel,
        "config": args.config,
        "source": args.source or f"{args.root} (tools/pmc.sh)",
        "fetch_size_bytes_raw": s["FETCH_SIZE"] * 1024.0,
        "hbm_bytes_per_launch": s["FETCH_SIZE"] * 1024.0 * 2.0,
        "correction": "x1024 (KiB) x2: gfx950 FETCH_SIZE counts 64-B halves of 128-B requests "
                      "(MI355X_MICROARCH.md HBM); WRITE_SIZE not collected (output 8.3 MB)",
    }
    if s.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
        out["l1_hit"] = 1.0 - s.get("TCP_TCC_READ_REQ_sum", 0.0) / s["TCP_TOTAL_CACHE_ACCESSES_sum"]
    if s.get("TCC_HIT_sum") is not None and s.get("TCC_MISS_sum") is not None:
        out["l2_hit"] = s["TCC_HIT_sum"] / max(1.0, s["TCC_HIT_sum"] + s["TCC_MISS_sum"])
    if s.get("SQ_WAVE_CYCLES"):
        if "SQ_WAIT_ANY" in s:
            out["sq_wait_any_frac"] = s["SQ_WAIT_ANY"] / s["SQ_WAVE_CYCLES"]
        if "SQ_ACTIVE_INST_ANY" in s:
            out["sq_active_frac"] = s["SQ_ACTIVE_INST_ANY"] / s["SQ_WAVE_CYCLES"]
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "TA_BUSY_avr", "SQ_WAVES",
              "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM", "SQ_BUSY_CU_CYCLES"):
        if k in s:
            out[k] = s[k]
    text = json.dumps(out, indent=1)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")
    if args.merge:
        allj = {"configs": {}}
        if os.path.exists(args.merge):
            with open(args.merge) as f:
                allj = json.load(f)
        allj.setdefault("configs", {})[args.config] = out
        with open(args.merge, "w") as f:
            f.write(json.dumps(allj, indent=1) + "\n")


if __name__ == "__main__":
    main()
