#!/usr/bin/env python3
"""Heavy tiles vs heavy pixels (analysis aid, not part of the product).

From the oracle's per-pixel, per-bounce visit profile (simd_model.profile),
with 32x2 lockstep tiles: a tile's lockstep cost is the sum over bounces of
its lanes' maximum visits; a pixel's cost is its own visits.  The bulk
estimate is the total lockstep cost over CUs x 24 resident waves (the
runtime's learn_order).  Prints the heaviest tiles' pixel costs and, for a few
pixel bars, how many pixels would be split and how long the longest remaining
tile wave would be.  Usage: heavy_pixel_model.py [config] [row step]
"""
import os
import sys

import numpy as np

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__))]
from simd_model import profile  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n_cu = 256
    vis, _, c = profile(k, 1, 1)
    H, W, B = vis.shape
    t = vis[: H // 2 * 2, : W // 32 * 32].reshape(H // 2, 2, W // 32, 32, B).transpose(0, 2, 1, 3, 4)
    t = t.reshape(-1, 64, B).astype(np.int64)
    lock = t.max(axis=1).sum(axis=1)
    px = t.sum(axis=2)
    order = np.argsort(lock)[::-1]
    bulk = lock.sum() / (n_cu * 24)
    print(f"config {k}: {len(lock)} tiles, total lockstep {lock.sum()}, bulk estimate {bulk:.0f} per slot; {c}")
    for r in (0, 1, 2, 5, 10, 20, 50, 72, 100, 200, 500, 1000):
        if r >= len(order):
            break
        i = order[r]
        p = np.sort(px[i])[::-1]
        print(f"  rank {r}: tile cost {lock[i]} ({lock[i] / bulk:.2f} x bulk), top pixels {p[:6].tolist()}, "
              f"{int((px[i] > bulk).sum())} over the bulk, {int((px[i] > 0.5 * bulk).sum())} over half")
    for f in (1.0, 0.75, 0.5):
        heavy = px > f * bulk
        t2 = t.copy()
        t2[heavy] = 0
        lock2 = t2.max(axis=1).sum(axis=1)
        print(f"  bar {f:.2f} x bulk: {int(heavy.sum())} heavy pixels in {int(heavy.any(axis=1).sum())} tiles; "
              f"longest remaining tile {lock2.max()} ({lock2.max() / bulk:.2f} x bulk), {int((lock2 > bulk).sum())} "
              f"tiles over the bulk")


if __name__ == "__main__":
    main()
