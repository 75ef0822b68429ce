"""Option accel, step 1 of VERDICT r04 "Next round" item 1: a CPU study.

For each BASELINE configuration it renders, on the CPU, the frame through
  * the oracle (oracle/rt_oracle.c: the reference's stack DFS over the
    reference's median-split, random-axis tree, here seeded with axis_seed 1),
  * the same oracle over the reference trees of other axis seeds (the
    reference's own tree is random per build, BVHBuilder.java:53),
  * the accel walk's CPU model (oracle/rt_accel_model.c) over the records
    rt_accel_records builds (1 layout and 8 octant layouts),
and records the pixels that differ from the seed-1 oracle frame (RGBA8 and
the float radiance's bits), node visits and triangle tests per segment, and
the lockstep cost: the sum over 8x8 tiles and bounces of the tile's longest
walk (what a wave of the GPU kernel steps through).

Output: tests/golden/accel_study.json (tests/test_accel_model.py checks the
claims it makes on small cases; DESIGN.md §4a cites it).

    python tools/accel_study.py [--quick]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-ray-tracer-vulkan_amd")]

import numpy as np  # noqa: E402

from oracle import oracle_lib as O  # noqa: E402
from rtamd import _lib, configs  # noqa: E402


def lockstep(prof: np.ndarray, tw: int = 8, th: int = 8):
    """(wave steps, lane steps) of 8x8 tiles from a per-pixel, per-bounce visit profile."""
    v = (prof & 0xFFFFF).astype(np.int64)
    R, W, B = v.shape
    v = v[: R // th * th, : W // tw * tw].reshape(R // th, th, W // tw, tw, B)
    return int(v.max(axis=(1, 3)).sum()), int(v.sum())


def diff(a_rgba, a_rad, b_rgba, b_rad):
    return {"rgba_px": int((a_rgba != b_rgba).any(-1).sum()),
            "radiance_px": int((a_rad.view(np.uint32) != b_rad.view(np.uint32)).any(-1).sum())}


def work(c: dict, prof: np.ndarray, row_step: int) -> dict:
    d = {"segments": c["segments"], "node_visits": c["node_visits"], "tri_tests": c["tri_tests"],
         "visits_per_segment": round(c["node_visits"] / max(1, c["segments"]), 3),
         "tri_tests_per_segment": round(c["tri_tests"] / max(1, c["segments"]), 3)}
    if row_step == 1:
        ws, ls = lockstep(prof)
        d["lockstep_wave_steps"] = ws
        d["lockstep_lane_util"] = round(ls / (64.0 * ws), 4) if ws else 0.0
    return d


def study(k: int, row_step: int, seeds, max_bounces=None) -> dict:
    cfg = configs.get(k)
    mb = max_bounces or cfg.max_bounces
    t0 = time.time()
    base = cfg.build(axis_seed=1)
    cam = cfg.camera()
    tile = (0, 0, cfg.width, cfg.height)
    ref = O.render_profile(base.model_vertex_data, base.model_material_data, base.flat_bvh_data, cam.ubo_bytes(),
                           cfg.width, cfg.height, mb, tile=tile, row_step=row_step)
    out = {"config": cfg.name, "width": cfg.width, "height": cfg.height, "max_bounces": mb,
           "row_step": row_step, "pixels": int(ref[0].shape[0] * ref[0].shape[1]),
           "reference_seed1": work(ref[2], ref[3], row_step), "reference_other_seeds": {}, "accel": {}}
    for s in seeds:
        b = cfg.build(axis_seed=s)
        r = O.render_profile(b.model_vertex_data, b.model_material_data, b.flat_bvh_data, cam.ubo_bytes(),
                             cfg.width, cfg.height, mb, tile=tile, row_step=row_step)
        e = work(r[2], r[3], row_step)
        e.update(diff(r[0], r[1], ref[0], ref[1]))
        e["segments_equal"] = r[2]["segments"] == ref[2]["segments"]
        out["reference_other_seeds"][str(s)] = e
    for nl in (1, 8):
        rec, info = _lib.accel_records(base, nl)
        a = O.render_accel(base.model_vertex_data, base.model_material_data, base.flat_bvh_data, cam.ubo_bytes(),
                           cfg.width, cfg.height, mb, rec, info, tile=tile, row_step=row_step, profile=True)
        e = work(a[2], a[3], row_step)
        e.update(diff(a[0], a[1], ref[0], ref[1]))
        e["segments_equal"] = a[2]["segments"] == ref[2]["segments"]
        e["mat_reads_equal"] = a[2]["mat_reads"] == ref[2]["mat_reads"]
        e["fallback_segments"] = a[2]["fallbacks"]
        e.update({"slots": info["slots"], "record_mb": round(rec.nbytes / 2**20, 2), "prims": info["n_prims"],
                  "reference_leaves": info["n_inputs"], "depth": info["depth"]})
        out["accel"][f"layouts{nl}"] = e
    if k in (3, 6):
        # the box margin's cost: the same walk with t_enter <= closest_t exactly
        from oracle.oracle_lib import lib as olib
        rec, info = _lib.accel_records(base, 1)
        olib(accel=True).orc_accel_margin(1.0, 0.0)
        try:
            a = O.render_accel(base.model_vertex_data, base.model_material_data, base.flat_bvh_data,
                               cam.ubo_bytes(), cfg.width, cfg.height, mb, rec, info, tile=tile, row_step=row_step)
        finally:
            olib(accel=True).orc_accel_margin(1.0 + 2.0**-10, 2.0**-10)
        e = {"visits_per_segment": round(a[2]["node_visits"] / a[2]["segments"], 3),
             "fallback_segments": a[2]["fallbacks"]}
        e.update(diff(a[0], a[1], ref[0], ref[1]))
        out["accel"]["layouts1_no_margin"] = e
    out["seconds"] = round(time.time() - t0, 1)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="configs 1-2 only")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "accel_study.json"))
    args = ap.parse_args()
    plan = [(1, 1, (2, 3), None), (2, 1, (2, 3), None), (2, 1, (2,), 10)]
    if not args.quick:
        plan += [(3, 1, (2, 3), None), (4, 1, (2,), None), (6, 1, (2, 3), None), (5, 16, (2,), None)]
    res = []
    for k, rs, seeds, mb in plan:
        r = study(k, rs, seeds, mb)
        print(json.dumps(r), flush=True)
        res.append(r)
    doc = {"what": "option accel CPU study (tools/accel_study.py): pixel differences from the seed-1 reference-order "
                   "oracle frame, and work per segment, for the reference tree under other axis seeds and for the "
                   "accel walk's model over 1 and 8 layouts",
           "cases": res}
    if not args.quick:
        with open(args.out, "w") as f:
            json.dump(doc, f, indent=1)
        print("wrote", args.out)


if __name__ == "__main__":
    main()
