#!/usr/bin/env python3
"""Per-wave timeline of the simple trace kernel (diagnostic build, option diag=1).

Prints: kernel span, wave duration percentiles, resident waves per CU over
time (mean / max), the tail (time during which fewer than half the CUs are
busy), and per-XCD totals.  Also saves the raw records to --out (npz)."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--bounces", type=int, default=0)
    ap.add_argument("--wave-tile", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/diag.npz")
    ap.add_argument("--opt", action="append", default=[], help="rt_set_option name=value (repeatable)")
    args = ap.parse_args()
    import torch
    import rtamd
    from rtamd import configs
    from rtamd._lib import check

    cfg = configs.get(args.config)
    built = cfg.build()
    cam = cfg.camera()
    W, H, B = cfg.width, cfg.height, (args.bounces or cfg.max_bounces)
    r = rtamd.Renderer((0,))
    r.upload_scene(built)
    r.set_option("kernel", 0)
    r.set_option("wave_tile", args.wave_tile)
    for kv in args.opt:
        k, v = kv.split("=")
        r.set_option(k, int(v))
    L = rtamd.lib()
    out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda:0")
    for diag in (0, 0, 1):
        r.set_option("diag", diag)
        r.render_tile_device(cam, W, H, B, 0, 0, W, H, out.data_ptr(), None, None)
    torch.cuda.synchronize()
    n = C.c_size_t()
    check(L.rt_diag_copy(r._ctx, None, 0, C.byref(n)))
    rec = np.zeros(n.value, dtype=np.uint64)
    check(L.rt_diag_copy(r._ctx, rec.ctypes.data, n.value, C.byref(n)))
    rec = rec.reshape(-1, 8)
    is_help = (rec[:, 2] >> 32) == 0xFFFFFFFF
    help_rec, rec = rec[is_help], rec[~is_help]
    t0, t1 = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64)
    hw, xcc = (rec[:, 2] & 0xFFFFFFFF).astype(np.int64), (rec[:, 2] >> 32).astype(np.int64)
    base = t0.min()
    t0, t1 = t0 - base, t1 - base
    span = t1.max()
    dur = t1 - t0
    cu = xcc * 256 + ((hw >> 8) & 0xFF)          # cu_id | sh | se bits
    print(f"waves {len(rec)}  span {span / 100:.1f} us (100 MHz ticks)  distinct CUs {len(np.unique(cu))}")
    print("wave duration us: p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f mean %.1f" % tuple(
        np.percentile(dur, [10, 50, 90, 99, 100]).tolist() + [dur.mean()]) if False else
        "wave duration us: p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f" % tuple(
            (np.percentile(dur, [10, 50, 90, 99, 100]) / 100).tolist()))
    # resident waves per CU over time
    grid = np.linspace(0, span, 200)
    ucu, inv = np.unique(cu, return_inverse=True)
    res = np.zeros((len(ucu), len(grid)))
    for k in range(len(rec)):
        a, b = np.searchsorted(grid, [t0[k], t1[k]])
        res[inv[k], a:b] += 1
    tot = res.sum(axis=0)
    busy = (res > 0).sum(axis=0)
    print("resident waves/CU (mean over CUs) at 10 time points:",
          " ".join(f"{x:.1f}" for x in (tot / len(ucu))[::20]))
    print("max resident waves on one CU:", int(res.max()))
    half = np.nonzero(busy < len(ucu) / 2)[0]
    if len(half):
        print(f"tail: fewer than half the CUs busy from {grid[half[0]] / 100:.1f} us to end ({span / 100:.1f} us)")
    print("per-XCD wave-time share:", [round(float(dur[xcc == x].sum() / dur.sum()), 3) for x in range(8)])
    print("first start / last start / last end (us):", 0, t0.max() / 100, span / 100)
    ends = np.sort(t1)
    print("time by which 50/90/99/99.9/100% of waves ended (us):",
          " ".join(f"{ends[min(len(ends) - 1, int(q * len(ends)))] / 100:.1f}" for q in (0.5, 0.9, 0.99, 0.999, 1.0)))
    alive = [int(((t0 <= g) & (t1 > g)).sum()) for g in grid[::10]]
    print("waves alive at 20 time points:", alive)
    blk = (rec[:, 3] >> 8).astype(np.int64)
    late = np.argsort(t1)[-20:]
    print("last 20 waves to finish: block ids", blk[late].tolist(), "durations us", (dur[late] / 100).astype(int).tolist())
    iters, wins, coop_t = rec[:, 4].astype(np.int64), rec[:, 5].astype(np.int64), rec[:, 6].astype(np.int64)
    print("lockstep iterations per wave: p50 %d p99 %d max %d; coop windows p50 %d max %d" % (
        np.median(iters), np.percentile(iters, 99), iters.max(), np.median(wins), wins.max()))
    for k in late[::-1][:8]:
        lock_t = max(1, dur[k] - coop_t[k])
        print(f"  slow wave block {blk[k]}: {dur[k] / 100:.0f} us, {iters[k]} lockstep iters "
              f"({lock_t / 100 / max(1, iters[k]) * 1000:.0f} ns each incl. shading), "
              f"{wins[k]} coop windows in {coop_t[k] / 100:.0f} us")
    lane_steps = rec[:, 7].astype(np.int64)          # word 7: the lanes' own lockstep steps, summed
    if iters.sum() > 0:
        print(f"lockstep lane utilisation: {lane_steps.sum() / (64.0 * iters.sum()):.3f} "
              f"({lane_steps.sum()} lane-steps over {iters.sum()} wave-steps)")
    if len(help_rec):
        hs, he = (help_rec[:, 0].astype(np.int64) - base) / 100, (help_rec[:, 1].astype(np.int64) - base) / 100
        rays = help_rec[:, 4].astype(np.int64)
        first = help_rec[:, 6].astype(np.int64)
        busy = rays > 0
        print(f"helper waves {len(help_rec)}: start p0 {hs.min():.0f} p50 {np.median(hs):.0f} us; end max {he.max():.0f} us; "
              f"rays total {rays.sum()} (waves with work {busy.sum()}, max per wave {rays.max()})")
        if busy.any():
            ft = (first[busy] - base) / 100
            print(f"  first ray taken at us p0 {ft.min():.0f} p50 {np.median(ft):.0f}; busy helpers end p50 {np.median(he[busy]):.0f} max {he[busy].max():.0f}")
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    np.savez(args.out, rec=rec)


if __name__ == "__main__":
    main()
