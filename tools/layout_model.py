#!/usr/bin/env python3
"""L2 traffic model of walk-record storage layouts (analysis aid, not part of
the product).

The oracle's exact visit sequences (orc_trace_pixel) of the 8x8 tile waves one
XCD traces (raster tile order, tile k on XCD k mod 8) in a band of tile rows
are replayed in lockstep (step k = every lane's k-th visit of its whole path);
`resident` waves run at once and each step's 128-B lines go through a 4 MB,
16-way LRU cache (tools/layout_sim.c).  Misses x 128 B approximate what the
XCD's L2 fetches (FETCH_SIZE); the layouts differ only in where the records
sit, so the visit sequence, and with it every counter, is the same.

Layouts (32-B slots, 4 per line):
  inline        the default walk records: preorder, a leaf's two slots inline
  inline_align  option leaf_align: a pad slot so no leaf straddles two lines
  split         preorder boxes, one slot per node, and the triangles in a
                second array at the node's own index (a sparse 32-B record)
  split_compact the same with the triangles packed by leaf ordinal
  separate      round 3's records: a 32-B box per node, a 48-B triangle
                record per leaf by leaf ordinal

The walk is replayed as the kernel runs it: bounce by bounce (the bounce loop
is wave-uniform), lockstep while two or more lanes walk, then the cooperative
tail (--coop 1, coop_lanes 1): the last lane's remaining visits in 64-slot
windows.  Config 5 (rows 103-166, 3,840 tiles of XCD 0): 292,630 windows, i.e.
9.9 M per frame (the GPU's diagnostic launch counts 9.48 M); the misses scale to
~20 GB per frame (PMC FETCH 28.5 GB), two thirds of them the windows', which
serve 4.2 visits each (median 2) and use 2.5 of their ~17 lines.

Usage: layout_model.py [--config 5] [--rows 64] [--row0 N] [--xcd 0] [--resident 1024] [--workers 8] [--coop 1]
"""
import argparse
import ctypes as C
import multiprocessing as mp
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-ray-tracer-vulkan_amd"), ROOT]

G = {}


def _init(k):
    from rtamd import configs
    from oracle import oracle_lib
    cfg = configs.get(k)
    b = cfg.build()
    L = oracle_lib.lib()
    L.orc_trace_pixel.restype = C.c_int
    L.orc_trace_pixel.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                  C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]
    G.update(cfg=cfg, b=b, L=L, cam=np.frombuffer(cfg.camera().ubo_bytes(), np.uint8).copy(),
             buf=np.zeros(1 << 18, dtype=np.int32))


def tile_steps(t):
    """The steps of tile t = (tx, ty), bounce by bounce as the kernel's
    wave-uniform bounce loop: the distinct nodes of each lockstep step while
    two or more lanes walk, then (cooperative tail) the last lane's remaining
    visits as windows, each entry -(x + 1) = a window starting at node x (the
    window's extent depends on the layout: tools/layout_sim.c)."""
    tx, ty = t
    cfg, b, L, buf = G["cfg"], G["b"], G["L"], G["buf"]
    W, H, B = cfg.width, cfg.height, cfg.max_bounces
    v, m, n = b.model_vertex_data, b.model_material_data, b.flat_bvh_data
    segs = [[] for _ in range(B)]
    for q in range(64):
        px, py = tx * 8 + (q & 7), ty * 8 + (q >> 3)
        if px >= W or py >= H:
            continue
        cnt = L.orc_trace_pixel(v.ctypes.data, v.nbytes, m.ctypes.data, m.nbytes, n.ctypes.data, n.nbytes,
                                G["cam"].ctypes.data, W, H, B, px, py, buf.ctypes.data, buf.size)
        s = buf[:max(cnt, 0)].copy()
        starts = np.flatnonzero(s < 0)
        for si, st in enumerate(starts[:B]):
            en = starts[si + 1] if si + 1 < len(starts) else len(s)
            if en > st + 1:
                segs[si].append(s[st + 1:en])
    counts, nodes = [], []
    coop, slot = G["coop"], G["slot"]
    for lanes in segs:
        if not lanes:
            continue
        lens = np.array([len(x) for x in lanes])
        mx = int(lens.max())
        # lockstep while two or more lanes walk (coop on: the last lane then
        # finishes in windows)
        srt = np.sort(lens)
        k_lock = int(srt[-2]) if (coop and len(lens) > 1) else (0 if coop else mx)
        M = np.full((len(lanes), max(k_lock, 1)), -1, np.int32)
        for i, x in enumerate(lanes):
            M[i, :min(len(x), k_lock)] = x[:k_lock]
        M = M[:, :k_lock]
        if k_lock > 0:
            M.sort(axis=0)
            keep = M >= 0
            keep[1:] &= M[1:] != M[:-1]
            counts.append(keep.sum(axis=0).astype(np.int64))
            nodes.append(M.T[keep.T])
        if coop and mx > k_lock:
            tail = lanes[int(np.argmax(lens))][k_lock:]
            win, ws = [], None
            for x in tail:
                if ws is None or not (ws <= slot[x] < ws + 63):
                    ws = slot[x]
                    win.append(-(int(x) + 1))
            counts.append(np.ones(len(win), np.int64))
            nodes.append(np.array(win, np.int32))
    if not counts:
        return np.zeros(0, np.int64), np.zeros(0, np.int32)
    return np.concatenate(counts), np.concatenate(nodes).astype(np.int32)


def layouts(nodes_i32):
    n = nodes_i32.shape[0]
    leaf = nodes_i32[:, 9] < 0
    out = {}
    nl = np.where(leaf, 2, 1)
    slot = np.concatenate([[0], np.cumsum(nl)[:-1]])
    lines = np.full((n, 3), -1, np.int64)
    lines[:, 0] = slot // 4
    lines[leaf, 1] = (slot[leaf] + 1) // 4
    out["inline"] = (lines, slot)
    # leaf_align: as rt_upload_scene
    slot2 = np.zeros(n, np.int64)
    s = 0
    for i in range(n):
        if leaf[i] and s % 4 == 3:
            s += 1
        slot2[i] = s
        s += 2 if leaf[i] else 1
    lines = np.full((n, 3), -1, np.int64)
    lines[:, 0] = slot2 // 4
    lines[leaf, 1] = (slot2[leaf] + 1) // 4
    out["inline_align"] = (lines, slot2)
    big = 1 << 40
    idx = np.arange(n, dtype=np.int64)
    lines = np.full((n, 3), -1, np.int64)
    lines[:, 0] = idx // 4
    lines[leaf, 1] = big + idx[leaf] // 4
    out["split"] = (lines, idx)
    ordl = np.cumsum(leaf) - 1
    lines = np.full((n, 3), -1, np.int64)
    lines[:, 0] = idx // 4
    lines[leaf, 1] = big + ordl[leaf] // 4
    out["split_compact"] = (lines, idx)
    lines = np.full((n, 3), -1, np.int64)
    lines[:, 0] = idx // 4
    b0 = ordl[leaf] * 48
    lines[leaf, 1] = big + b0 // 128
    lines[leaf, 2] = np.where((b0 + 47) // 128 != b0 // 128, big + (b0 + 47) // 128, -1)
    out["separate"] = (lines, idx)
    # dedupe the second / third line where it equals the first
    for k, (l, _) in out.items():
        l[:, 1] = np.where(l[:, 1] == l[:, 0], -1, l[:, 1])
        l[:, 2] = np.where((l[:, 2] == l[:, 0]) | (l[:, 2] == l[:, 1]), -1, l[:, 2])
        # compact: -1 holes before valid entries
        bad = (l[:, 1] < 0) & (l[:, 2] >= 0)
        l[bad, 1], l[bad, 2] = l[bad, 2], -1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--rows", type=int, default=64, help="tile rows of the band")
    ap.add_argument("--row0", type=int, default=-1, help="first tile row (default: the band centred)")
    ap.add_argument("--xcd", type=int, default=0)
    ap.add_argument("--resident", type=int, default=1024)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--l2-mb", type=float, default=4.0)
    ap.add_argument("--coop", type=int, default=1, help="1 = the cooperative tail (coop_lanes 1), 0 = off")
    args = ap.parse_args()
    so = os.path.join("/tmp", "liblayout_sim.so")
    subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tools", "layout_sim.c")])
    sim = C.CDLL(so)
    sim.layout_sim.restype = C.c_int64
    sim.layout_sim.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                               C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int64)]
    _init(args.config)
    nd = np.frombuffer(G["b"].flat_bvh_data.tobytes(), dtype=np.int32).reshape(-1, 12)
    L = layouts(nd)
    G["coop"] = args.coop
    G["slot"] = L["inline"][1]
    cfg = G["cfg"]
    tiles_x, tiles_y = (cfg.width + 7) // 8, (cfg.height + 7) // 8
    row0 = args.row0 if args.row0 >= 0 else max(0, (tiles_y - args.rows) // 2)
    tiles = [(k % tiles_x, k // tiles_x) for k in range(row0 * tiles_x, min(tiles_y, row0 + args.rows) * tiles_x)
             if k % 8 == args.xcd]
    t0 = time.time()
    with mp.get_context("fork").Pool(args.workers) as pool:
        res = pool.map(tile_steps, tiles, chunksize=8)
    t1 = time.time()
    counts = np.concatenate([r[0] for r in res])
    nodes = np.concatenate([r[1] for r in res])
    tile_ptr = np.concatenate([[0], np.cumsum([len(r[0]) for r in res])]).astype(np.int64)
    step_ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    ways = 16
    sets = int(args.l2_mb * 1024 * 1024 / 128 / ways)
    print(f"config {args.config}: XCD {args.xcd}, tile rows {row0}-{row0 + args.rows - 1}, {len(tiles)} tiles, "
          f"{len(counts)} wave steps, {len(nodes)} node accesses, traced in {t1 - t0:.0f} s; "
          f"L2 {args.l2_mb} MB ({sets} sets x {ways}), {args.resident} resident waves, "
          f"coop windows {int((nodes < 0).sum())}")
    base = None
    for name, (lines, nslot) in L.items():
        acc = C.c_int64(0)
        nslot = np.ascontiguousarray(nslot, dtype=np.int64)
        miss = sim.layout_sim(len(res), tile_ptr.ctypes.data, step_ptr.ctypes.data, nodes.ctypes.data,
                              lines.ctypes.data, nslot.ctypes.data, len(nslot), 64, args.resident, sets, ways,
                              C.byref(acc))
        base = base or miss
        print(f"  {name:14s} line accesses {acc.value:12d}  misses {miss:11d}  ({miss * 128 / 1e6:9.1f} MB, "
              f"{miss / base:.3f} x inline)")


if __name__ == "__main__":
    main()
