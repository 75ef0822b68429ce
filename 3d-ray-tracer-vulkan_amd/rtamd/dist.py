"""Multi-GPU frame tiling: one process per GPU (torch.distributed; backend
"nccl" = RCCL over xGMI on MI355X, "gloo" for CPU tests).

Partitions of a frame over the N ranks:

* contiguous spans of an exchange batch (bench.py's N > 1 default since round
  5; SpanPlan, SpanTracer, span_send / span_post_recvs / span_finish_recvs,
  exchange_spans): a batch of G frames is one column of G x H rows cut into N
  contiguous spans of whole bands, rank 0's root_weight times the others'; a
  rank traces its span one frame per launch (whole frames, a band run at either
  end) and rank 0 receives every other span straight into the batch's frames
  (RCCL point-to-point, no assembly); optionally the rows travel as RGB (3/4
  of the bytes; the alpha byte is always 255; wire_copy);
* weighted interleaved row bands (round 4's default; band_owners,
  SharePlan, gather_shares): the band_h-row bands are dealt out by a smooth
  weighted round robin, rank 0 with weight root_weight (it also receives and
  assembles every frame) and the others with weight 1, so every rank's bands
  are spread over the frame; a rank traces its bands of a batch of frames in
  one launch (rt_render_batch_device), one gather per batch brings the
  packed bands to rank 0, which assembles the frames with one index_select.
  root_weight 1 is the plain interleave: rank r gets the bands b = r mod N
  (band_rows, gather_frame, gather_frames);
* rotating contiguous pieces (SharePlan layout "pieces"; bench.py --partition
  pieces, an option): the frame cut into N contiguous pieces of whole bands; in
  frame f rank r traces piece (r + f) mod N, and a launch of N consecutive
  frames (rt_render_batch_lists_device, one band list per frame) holds every
  piece once, each of a different frame, so every rank traces one whole
  frame's rows per step with a whole frame's spatial coherence; gathered and
  assembled like the bands;
* a tile grid (tile_grid, tile_rects, TilePlan, gather_tiles): N = gx x gy
  rectangles, e.g. BASELINE config 4's 2 x 2 over 4 GPUs; one gather of the
  (padded) tiles and one index_select;
* rotating row pieces (block_layout, exchange_blocks; an option, measured
  slower on the sending ranks): one contiguous run of rows per rank, laid out
  in an order that rotates every frame; rank 0 receives the others straight
  into the frame (RCCL point-to-point in one group);
* frame batches (BatchPlan, gather_batch; weak scaling): N frames per step,
  bands rotated.

Every gather can carry the RGBA8 frame and, beside it, the float radiance
(the sqrt'd colour before quantisation, 3 floats per pixel), which the north
star's "RCCL gather of per-tile radiance buffers" names.  The scene is
replicated on every rank (uploaded once per rank); pixels are independent and
seeded by their global (x, y) (compute_dynamic_ray.comp:164), so every
partition's frame equals the one-GPU frame bit for bit.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Optional

import numpy as np

from ._lib import check, lib


def band_row_count(height: int, band_h: int, world: int, rank: int) -> int:
    n = lib().rt_band_rows(height, band_h, world, rank)
    if n < 0:
        raise ValueError("bad band partition")
    return n


def band_rows(height: int, band_h: int, world: int, rank: int) -> np.ndarray:
    """Frame rows of rank's bands, in the packed order the kernels write them."""
    y = np.arange(height)
    return y[(y // band_h) % world == rank]


def gather_frame(local, height: int, band_h: int, group=None):
    """Gather every rank's packed band rows (torch tensor [rows_r, W, C], or
    the padded [max_rows, W, C] buffer) to rank 0 and assemble the
    [height, W, C] frame there (None elsewhere).  A one-frame batch: one
    gather into a single stack and one index_select with a cached device
    index, so a step issues no host-to-device copy and never waits on the GPU."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    plan, src_index = _cached_plan(height, band_h, world, 1, local.device)
    if local.shape[0] < plan.max_rows:
        pad = torch.zeros((plan.max_rows - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        local = torch.cat([local, pad])
    elif local.shape[0] > plan.max_rows:
        local = local[: plan.max_rows]
    out = gather_batch(local.unsqueeze(0), plan, group, src_index=src_index)
    return None if out is None else out[0]


def gather_frames(local, height: int, band_h: int, group=None):
    """Several one-frame steps of the bands partition gathered at once:
    local is this rank's [n_frames, max_rows, W, C] packed bands of n_frames
    frames (rank r traced the bands r of each); returns the
    [n_frames, height, W, C] frames on rank 0, None elsewhere.  One collective
    and one index_select for the whole batch, so the per-frame host cost of
    the exchange shrinks with the batch."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    plan, src_index = _cached_plan(height, band_h, world, local.shape[0], local.device, rotate=False)
    if local.shape[1] != plan.max_rows:
        raise ValueError(f"gather_frames: {local.shape[1]} rows per frame, the partition packs {plan.max_rows}")
    return gather_batch(local, plan, group, src_index=src_index)


# --- weighted interleaved bands, batched (bench.py's N > 1 default) --------


def band_owners(height: int, band_h: int, world: int, root_weight: float = 1.0) -> np.ndarray:
    """Owner rank of every band_h-row band of the frame: a smooth weighted
    round robin (each band goes to the rank with the largest running credit;
    credits grow by the rank's weight and the winner pays the total), rank 0
    weighted root_weight and the others 1, ties to the lower rank.  Every
    rank's bands are spread over the whole frame, in proportion to its weight;
    root_weight 1 gives band b to rank b mod world."""
    n = (height + band_h - 1) // band_h
    w = np.ones(world, np.float64)
    w[0] = max(0.0, float(root_weight))
    total = w.sum()
    credit = np.zeros(world, np.float64)
    owner = np.empty(n, np.int64)
    for b in range(n):
        credit += w
        r = int(np.argmax(credit))          # first maximum: the lower rank wins ties
        owner[b] = r
        credit[r] -= total
    return owner


def dealt_bands(height: int, band_h: int, world: int, root_weight: float = 1.0) -> list:
    """The weighted round robin of band_owners run on over world consecutive
    frames (the credits carry from one frame into the next): table[f][r] is
    rank r's bands of frame f mod world.  Within a frame a rank's count
    differs from its weighted share by under a band, as with band_owners; over
    the world frames every rank's total is within one band of
    world x its share, so a launch of world frames (weak scaling) gives every
    rank other than 0 the same work to a band, where a fixed deal gives some
    of them a whole band per frame more (at 1080 rows, N = 8, root weight
    0.8: 18 bands to ranks 1-2, 17 to ranks 3-7)."""
    n = (height + band_h - 1) // band_h
    w = np.ones(world, np.float64)
    w[0] = max(0.0, float(root_weight))
    total = w.sum()
    credit = np.zeros(world, np.float64)
    table = []
    for _ in range(world):
        owner = np.empty(n, np.int64)
        for b in range(n):
            credit += w
            r = int(np.argmax(credit))
            owner[b] = r
            credit[r] -= total
        table.append([np.flatnonzero(owner == r).astype(np.int32) for r in range(world)])
    return table


def band_list(height: int, band_h: int, world: int, rank: int, root_weight: float = 1.0) -> np.ndarray:
    """rank's band indices, increasing (rt_render_batch_device's list)."""
    return np.flatnonzero(band_owners(height, band_h, world, root_weight) == rank).astype(np.int32)


def list_rows(height: int, band_h: int, bands) -> np.ndarray:
    """Frame rows of a band list, in the packed order the kernel writes them."""
    bands = np.asarray(bands, np.int64)
    if len(bands) == 0:
        return np.zeros(0, np.int64)
    rows = (bands[:, None] * band_h + np.arange(band_h)[None, :]).reshape(-1)
    return rows[rows < height]


def piece_owners(height: int, band_h: int, world: int) -> np.ndarray:
    """Owner position of every band_h-row band when the frame is cut into
    world contiguous pieces of whole bands (sizes differ by at most one band):
    piece p holds the bands [floor(p * n / world), floor((p + 1) * n / world))."""
    n = (height + band_h - 1) // band_h
    return (np.arange(n) * world) // n if n else np.zeros(0, np.int64)


def weighted_pieces(height: int, band_h: int, world: int, frame: int, root_weight: float):
    """Frame `frame`'s contiguous pieces, rank by rank (band index arrays):
    position p belongs to rank (p - frame) mod world; rank 0's piece has
    round(root_weight x n / (world - 1 + root_weight)) of the n bands, the
    other ranks share the rest as evenly as whole bands allow (the earlier
    positions one band more)."""
    n = (height + band_h - 1) // band_h
    s0 = int(round(max(0.0, root_weight) * n / (world - 1 + max(0.0, root_weight)))) if world > 1 else n
    s0 = min(s0, n)
    rest = n - s0
    sizes, k = [], 0
    for p in range(world):
        r = (p - frame) % world
        if r == 0:
            sizes.append(s0)
        else:
            sizes.append(rest // (world - 1) + (1 if k < rest % (world - 1) else 0))
            k += 1
    out = [None] * world
    b = 0
    for p in range(world):
        r = (p - frame) % world
        out[r] = np.arange(b, b + sizes[p], dtype=np.int32)
        b += sizes[p]
    return out


class SharePlan:
    """Row bookkeeping of a batch of n_frames frames over world ranks in
    weighted bands.  Rank r's exchange buffer holds its shares of the batch's
    frames back to back (frame f's rows at [off[r][f], off[r][f] + R), as
    rt_render_batch_device writes a batch of frames), padded to per_rank rows
    so that every rank sends the same size.

    rotate=False: rank r has the same bands in every frame (strong scaling,
    bench.py --partition bands).  rotate=True (weights 1 only): in frame f,
    rank r traces the bands of position (r + f) mod world, so over world
    frames every rank traces every band once.

    layout="pieces" (weak scaling, bench.py --partition pieces; rotates): the
    positions are world contiguous pieces of the frame (piece_owners), rank r
    tracing position (r + f) mod world in frame f, so a launch of world
    consecutive frames holds every piece once, each of a different frame: one
    whole frame's rows with a whole frame's spatial coherence.  With
    root_weight w < 1 rank 0's piece is w times the others' (weighted_pieces):
    the cut points then move with rank 0's piece from frame to frame, so over
    world frames a rank r > 0 covers every position with pieces of one size.
    Frames sit at a fixed stride of max_rows rows (off[r][f] = f * max_rows),
    as rt_render_batch_lists_device writes per-frame lists padded to the
    longest piece; launch_lists gives those lists.

    layout="dealt" (weak scaling, bench.py --partition bands --deal rotate):
    weighted interleaved bands dealt on over world frames (dealt_bands), one
    band list per frame, packed like the pieces (lists, max_rows stride)."""

    def __init__(self, height: int, band_h: int, world: int, n_frames: int, root_weight: float = 1.0,
                 rotate: bool = False, layout: str = "interleave"):
        if layout in ("pieces", "dealt"):
            rotate = True
        elif rotate and root_weight != 1.0:
            raise ValueError("rotating bands take equal weights")
        if layout not in ("interleave", "pieces", "dealt"):
            raise ValueError(f"unknown layout {layout!r}")
        # per-frame band lists (rt_render_batch_lists_device), frames at a max_rows stride
        self.lists = layout in ("pieces", "dealt")
        self.height, self.band_h, self.world, self.n_frames = height, band_h, world, n_frames
        self.root_weight, self.rotate, self.layout = root_weight, rotate, layout
        owner = piece_owners(height, band_h, world) if layout == "pieces" else \
            band_owners(height, band_h, world, root_weight)
        self.pos_bands = [np.flatnonzero(owner == r).astype(np.int32) for r in range(world)]
        self.pos_rows = [list_rows(height, band_h, b) for b in self.pos_bands]
        self.bands = self.pos_bands                    # rank r's bands (rotate=False)
        self.rows = self.pos_rows
        self.counts = [len(x) for x in self.pos_rows]
        # weighted pieces: rank r's bands in frame f (mod world), a table
        self.wtable = None
        if layout == "pieces" and root_weight != 1.0:
            self.wtable = [weighted_pieces(height, band_h, world, f, root_weight) for f in range(world)]
            self.counts = [len(list_rows(height, band_h, self.wtable[0][r])) for r in range(world)]
        elif layout == "dealt":
            self.wtable = dealt_bands(height, band_h, world, root_weight)
            # rows per frame, averaged over the world frames of the deal
            self.counts = [sum(len(list_rows(height, band_h, self.wtable[f][r])) for f in range(world)) // world
                           for r in range(world)]
        self.max_rows = max(len(self.frame_rows(r, f)) for r in range(world) for f in range(min(world, n_frames)))
        self.n_per = max(len(self.frame_bands(r, f)) for r in range(world) for f in range(min(world, n_frames)))
        self.off = [[0] * n_frames for _ in range(world)]
        self.per_rank = 0
        for r in range(world):
            o = 0
            for f in range(n_frames):
                self.off[r][f] = o
                o += self.max_rows if self.lists else len(self.frame_rows(r, f))
            self.per_rank = max(self.per_rank, o)
        src = np.empty(n_frames * height, np.int64)
        for r in range(world):
            for f in range(n_frames):
                rows = self.frame_rows(r, f)
                src[f * height + rows] = r * self.per_rank + self.off[r][f] + np.arange(len(rows))
        self.src = src

    def position(self, rank: int, frame: int) -> int:
        return (rank + frame) % self.world if self.rotate else rank

    def frame_bands(self, rank: int, frame: int) -> np.ndarray:
        if self.wtable is not None:
            return self.wtable[frame % self.world][rank]
        return self.pos_bands[self.position(rank, frame)]

    def frame_rows(self, rank: int, frame: int) -> np.ndarray:
        if self.wtable is not None:
            return list_rows(self.height, self.band_h, self.wtable[frame % self.world][rank])
        return self.pos_rows[self.position(rank, frame)]

    def launch_lists(self, rank: int, frame0: int, n: int) -> np.ndarray:
        """rt_render_batch_lists_device's bands for frames frame0 .. frame0 + n - 1
        of the batch: n lists of n_per entries, -1 padded."""
        out = np.full((n, self.n_per), -1, np.int32)
        for f in range(n):
            b = self.frame_bands(rank, frame0 + f)
            out[f, :len(b)] = b
        return out


_SHARE_PLANS: dict = {}


def cached_share_plan(height: int, band_h: int, world: int, n_frames: int, root_weight: float, device,
                      rotate: bool = False, layout: str = "interleave"):
    """SharePlan and its source-row index on `device`, built once per layout."""
    import torch
    key = (height, band_h, world, n_frames, float(root_weight), str(device), rotate, layout)
    hit = _SHARE_PLANS.get(key)
    if hit is None:
        plan = SharePlan(height, band_h, world, n_frames, root_weight, rotate, layout)
        hit = (plan, torch.as_tensor(plan.src, device=device))
        _SHARE_PLANS[key] = hit
    return hit


def gather_shares(local, plan: SharePlan, group=None, src_index=None, n_frames: int = None):
    """local: this rank's [per_rank, W, C] exchange buffer (its packed shares
    of the batch's frames, then padding).  One gather into a [world, ...]
    stack on rank 0 and one index_select; returns the [n_frames, height, W, C]
    frames on rank 0 (the first n_frames of the batch, default all), None
    elsewhere."""
    stack = gather_stack(local, plan, group)
    return None if stack is None else assemble_shares(stack, plan, src_index, n_frames)


def assemble_shares(stack, plan: SharePlan, src_index=None, n_frames: int = None):
    """Rank 0's frames from the gathered [world, per_rank, W, C] stack: one
    index_select (it may run on another stream than the gather)."""
    import torch
    if src_index is None:
        src_index = torch.as_tensor(plan.src, device=stack.device)
    n = plan.n_frames if n_frames is None else n_frames
    out = torch.index_select(stack.reshape(plan.world * plan.per_rank, -1), 0, src_index[: n * plan.height])
    return out.reshape((n, plan.height) + tuple(stack.shape[2:]))


def gather_stack(local, plan: SharePlan, group=None):
    """The gather half of gather_shares: every rank's buffer into one
    [world, per_rank, W, C] stack on rank 0 (None elsewhere)."""
    import torch
    import torch.distributed as dist
    if local.shape[0] != plan.per_rank:
        raise ValueError(f"gather_shares: {local.shape[0]} rows, the plan sends {plan.per_rank}")
    rank = dist.get_rank(group)
    stack = gl = None
    if rank == 0:
        stack = torch.empty((plan.world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
        gl = list(stack.unbind(0))
    if dist.get_backend(group) == "gloo" and local.is_cuda:       # gloo moves host memory
        host = local.cpu()
        hl = [torch.empty_like(host) for _ in range(plan.world)] if rank == 0 else None
        dist.gather(host, hl, dst=0, group=group)
        if rank == 0:
            for d, h in zip(gl, hl):
                d.copy_(h)
    else:
        dist.gather(local, gl, dst=0, group=group)
    return stack if rank == 0 else None


# --- a tile grid (BASELINE config 4: the screen tiled 2 x 2 over 4 GPUs) ----


def tile_grid(world: int):
    """(gx, gy) with gx * gy == world, as square as possible, gx >= gy
    (1 -> 1 x 1, 2 -> 2 x 1, 4 -> 2 x 2, 8 -> 4 x 2)."""
    gy = int(np.floor(np.sqrt(world)))
    while world % gy:
        gy -= 1
    return world // gy, gy


def tile_rects(width: int, height: int, gx: int, gy: int):
    """Rank r's rectangle (x0, y0, w, h), row-major over the grid; the
    remainder pixels go to the last column / row."""
    xs = [width * i // gx for i in range(gx + 1)]
    ys = [height * j // gy for j in range(gy + 1)]
    return [(xs[i], ys[j], xs[i + 1] - xs[i], ys[j + 1] - ys[j]) for j in range(gy) for i in range(gx)]


class TilePlan:
    """Pixel bookkeeping of n_frames frames over a tile grid: rank r sends
    [n_frames, hmax * wmax] pixels, frame f's tile packed at the start of its
    row (h x w, row pitch w: rt_render_tile_device's layout); src maps every
    frame pixel to its row in the gathered [world * n_frames * hmax * wmax]
    stack."""

    def __init__(self, width: int, height: int, world: int, n_frames: int = 1):
        self.width, self.height, self.world, self.n_frames = width, height, world, n_frames
        self.gx, self.gy = tile_grid(world)
        self.rects = tile_rects(width, height, self.gx, self.gy)
        self.hmax = max(r[3] for r in self.rects)
        self.wmax = max(r[2] for r in self.rects)
        self.tile_px = self.hmax * self.wmax
        per = n_frames * self.tile_px
        src = np.empty((n_frames, height, width), np.int64)
        for r, (x0, y0, w, h) in enumerate(self.rects):
            yy, xx = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
            for f in range(n_frames):
                src[f, y0:y0 + h, x0:x0 + w] = r * per + f * self.tile_px + yy * w + xx
        self.src = src.reshape(-1)


def gather_tiles(local, plan: TilePlan, group=None, src_index=None):
    """local: this rank's [n_frames, hmax * wmax, C] tiles (each packed at the
    start of its row).  Returns the [n_frames, height, width, C] frames on
    rank 0, None elsewhere."""
    stack = gather_tile_stack(local, plan, group)
    return None if stack is None else assemble_tiles(stack, plan, src_index)


def gather_tile_stack(local, plan: TilePlan, group=None):
    """The gather half of gather_tiles: every rank's tiles into one
    [world, n_frames, hmax * wmax, C] stack on rank 0 (None elsewhere)."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    stack = gl = None
    if rank == 0:
        stack = torch.empty((plan.world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
        gl = list(stack.unbind(0))
    if dist.get_backend(group) == "gloo" and local.is_cuda:
        host = local.cpu()
        hl = [torch.empty_like(host) for _ in range(plan.world)] if rank == 0 else None
        dist.gather(host, hl, dst=0, group=group)
        if rank == 0:
            for d, h in zip(gl, hl):
                d.copy_(h)
    else:
        dist.gather(local, gl, dst=0, group=group)
    return stack if rank == 0 else None


def assemble_tiles(stack, plan: TilePlan, src_index=None):
    """Rank 0's [n_frames, height, width, C] frames from the gathered tile
    stack: one index_select."""
    import torch
    if src_index is None:
        src_index = torch.as_tensor(plan.src, device=stack.device)
    c = stack.shape[-1]
    out = torch.index_select(stack.reshape(-1, c), 0, src_index)
    return out.reshape(plan.n_frames, plan.height, plan.width, c)


# --- one rank's launches (bench.py's trace) ----------------------------------


class ShareTracer:
    """The launches that trace one rank's share of frames, exactly as bench.py
    issues them (and as tests/test_gpu_dist.py replays them):

    * mode "whole": whole frames, n per launch (rt_render_batch_device, no list);
    * mode "bands" / "pieces" with a SharePlan: the rank's band list of each
      frame (one list for every frame of a launch, rt_render_batch_device; or
      one list per frame when plan.lists, rt_render_batch_lists_device), packed
      at plan.off[rank][f] of the rank's exchange buffer;
    * mode "tiles" with a TilePlan: the rank's rectangle of n frames in one
      launch (rt_render_batch_rect_device) when the rectangles are all the
      plan's tile size, else one rt_render_tile_device per frame, frame f's
      tile at f x tile_px of the buffers.

    Frame k of the run is frame k mod batch of the exchange batch (the plans'
    frame index).  Band lists are built once per (frame, count), so a launch
    does no host work beyond the ABI call."""

    def __init__(self, ctx, width: int, height: int, max_bounces: int, mode: str, rank: int = 0,
                 plan: Optional[SharePlan] = None, tplan: Optional[TilePlan] = None, band_h: int = 8,
                 batch: int = 1):
        if mode in ("bands", "pieces") and plan is None:
            raise ValueError(f"mode {mode!r} needs a SharePlan")
        if mode == "tiles" and tplan is None:
            raise ValueError("mode 'tiles' needs a TilePlan")
        if plan is not None and plan.lists and height % band_h:
            # rt_render_batch_lists_device packs whole bands at a fixed stride
            raise ValueError(f"per-frame band lists need band_h ({band_h}) to divide the height ({height})")
        self.ctx, self.W, self.H, self.B = ctx, width, height, max_bounces
        self.mode, self.rank, self.plan, self.tplan, self.band_h, self.G = mode, rank, plan, tplan, band_h, batch
        self.my_bands = [np.ascontiguousarray(plan.frame_bands(rank, f), dtype=np.int32) for f in range(batch)] \
            if plan is not None else None
        self.rect = tplan.rects[rank] if tplan is not None else None
        self._lists = {}

    @staticmethod
    def _i32p(a):
        return a.ctypes.data_as(C.POINTER(C.c_int32)) if a is not None else None

    def launch(self, cams, k0: int, n: int, stream: int, rgba_ptr, rad_ptr, stats=None) -> None:
        """Frames k0 .. k0 + n - 1 (cams: a ctypes array of their n CameraUBO)
        in one launch on `stream` (a HIP stream handle), into rgba_ptr /
        rad_ptr (device pointers; rad_ptr may be None); stats: an rt_stats or
        None."""
        L = lib()
        stp = C.byref(stats) if stats is not None else None
        if self.mode == "tiles":
            x0, y0, w, h = self.rect
            if n == 1 or w * h == self.tplan.tile_px:
                check(L.rt_render_batch_rect_device(self.ctx, cams, n, self.W, self.H, self.B, x0, y0, w, h,
                                                    rgba_ptr, rad_ptr, stream, stp))
            else:
                if stats is not None:
                    raise ValueError("stats of a multi-frame launch of unequal tiles")
                for f in range(n):
                    check(L.rt_render_tile_device(self.ctx, C.byref(cams[f]), self.W, self.H, self.B, x0, y0, w, h,
                                                  rgba_ptr + f * self.tplan.tile_px * 4,
                                                  (rad_ptr + f * self.tplan.tile_px * 12) if rad_ptr else None,
                                                  stream, None))
        elif self.plan is not None and self.plan.lists:
            key = (k0 % self.G, n)
            pl = self._lists.get(key)
            if pl is None:
                pl = self._lists[key] = np.ascontiguousarray(self.plan.launch_lists(self.rank, k0 % self.G, n))
            check(L.rt_render_batch_lists_device(self.ctx, cams, n, self.W, self.H, self.B, self.band_h,
                                                 self._i32p(pl), self.plan.n_per, rgba_ptr, rad_ptr, stream, stp))
        else:
            bl = self.my_bands[k0 % self.G] if self.my_bands is not None else None
            check(L.rt_render_batch_device(self.ctx, cams, n, self.W, self.H, self.B,
                                           self.band_h if bl is not None else 0, self._i32p(bl),
                                           len(bl) if bl is not None else 0, rgba_ptr, rad_ptr, stream, stp))

    def offset_rows(self, k0: int) -> int:
        """Bands / pieces: the row of the rank's exchange buffer where frame
        k0's share starts."""
        return self.plan.off[self.rank][k0 % self.G]


# --- contiguous spans of a batch (weak scaling; bench.py --partition spans) ---
#
# A batch of G frames is one column of G x H rows (frame f's rows at
# [f * H, (f + 1) * H)).  Rank r traces one contiguous span of it, cut at
# whole bands, rank 0's span root_weight times the others': whole frames where
# the span covers them, a run of bands of one frame at either end.  Whole
# frames are the kernel's most efficient launch (a band share of every frame
# traces ~20% slower per pixel, profiles/r05/r5k/emu), and the spans tile the
# batch column in rank order, so rank 0 receives every other span straight into
# the batch's frames (RCCL point-to-point in one group) and traces its own span
# in place: there is no stack and no assembly pass.


class SpanPlan:
    """Rank r's span of a batch of n_frames frames: bands [cuts[r],
    cuts[r + 1]) of the batch's n_frames * (height / band_h) bands, i.e. rows
    [row0[r], row0[r] + rows[r]) of the batch column.  launches[r] lists its
    launches: (frame, band_lo, band_hi, out_row), one frame each, the whole
    frame when (band_lo, band_hi) == (0, height / band_h), written at row
    out_row of the rank's span buffer (rank 0: the batch column from row0[0]).
    groups[r] lists the GPU launches over them: (first, count) runs of up to
    launch_frames consecutive entries of launches[r], traced in one launch
    (rt_render_batch_runs_device; one entry: rt_render_batch_device), their
    rows contiguous in the span buffer; pieces() follow the groups."""

    def __init__(self, height: int, band_h: int, world: int, n_frames: int, root_weight: float = 1.0,
                 whole_frames: bool = False, batch: int = 0, launch_frames: int = 1):
        if height % band_h:
            raise ValueError(f"spans: band_h ({band_h}) must divide the height ({height})")
        if not root_weight >= 0:
            raise ValueError("spans: root_weight must be >= 0")
        self.height, self.band_h, self.world, self.n_frames = height, band_h, world, n_frames
        self.root_weight = root_weight
        if not 1 <= launch_frames <= 16:
            raise ValueError("spans: launch_frames must be in 1..16")
        self.launch_frames = launch_frames
        self.whole_frames = whole_frames
        self.bpf = height // band_h
        total = n_frames * self.bpf
        if whole_frames:
            # cut at frame boundaries: every launch a whole frame (a band run
            # at a span's ends is a smaller launch that runs past its tail
            # less well); rank 0 its weighted share of frames rounded, the
            # other ranks the rest, the remainder's extra frames rotating over
            # them from batch to batch (batch: the batch's index)
            c = self.frame_counts(batch)
            self.cuts = [int(x) * self.bpf for x in np.concatenate([[0], np.cumsum(c)])]
        else:
            w = np.array([root_weight] + [1.0] * (world - 1))
            cum = np.concatenate([[0.0], np.cumsum(w)])
            self.cuts = [int(round(total * c / cum[-1])) for c in cum]
        self.cuts[-1] = total
        self.row0 = [c * band_h for c in self.cuts[:-1]]
        self.rows = [(self.cuts[r + 1] - self.cuts[r]) * band_h for r in range(world)]
        self.per_rank = max(self.rows)
        self.counts = [r // n_frames for r in self.rows]      # rows per frame, on average
        self.launches = []
        for r in range(world):
            out, b, out_row = [], self.cuts[r], 0
            while b < self.cuts[r + 1]:
                f = b // self.bpf
                lo = b - f * self.bpf
                hi = min(self.bpf, self.cuts[r + 1] - f * self.bpf)
                out.append((f, lo, hi, out_row))
                out_row += (hi - lo) * band_h
                b = f * self.bpf + hi
            self.launches.append(out)
        self.groups = [[(i, min(launch_frames, len(ls) - i)) for i in range(0, len(ls), launch_frames)]
                       for ls in self.launches]
        self._views = {}
        if whole_frames:
            # buffers hold the largest span of any batch
            self.per_rank = max(max(self.frame_counts(b)) for b in range(max(1, world - 1))) * height

    def frame_counts(self, batch: int):
        """whole_frames: the frames of each rank's span in batch `batch`."""
        if self.world == 1:
            return [self.n_frames]
        share = self.n_frames * self.root_weight / (self.root_weight + self.world - 1)
        g0 = min(self.n_frames, int(np.floor(share + 0.5)))
        q, m = divmod(self.n_frames - g0, self.world - 1)
        out = [g0] + [q] * (self.world - 1)
        for i in range(m):
            out[1 + (batch * m + i) % (self.world - 1)] += 1
        return out

    def batch(self, b: int) -> "SpanPlan":
        """The plan of batch b: this one, or with whole_frames the batch's own
        cut (its extra frames on other ranks); one object per distinct cut."""
        if not self.whole_frames or self.world <= 2:
            return self
        key = (b * ((self.n_frames - self.frame_counts(0)[0]) % (self.world - 1))) % (self.world - 1)
        v = self._views.get(key)
        if v is None:
            v = SpanPlan(self.height, self.band_h, self.world, self.n_frames, self.root_weight, True, b,
                         self.launch_frames)
            v.per_rank = self.per_rank
            self._views[key] = v
        return v

    def recv_slices(self):
        """(rank, row0, rows) of every span rank 0 receives."""
        return [(r, self.row0[r], self.rows[r]) for r in range(1, self.world) if self.rows[r] > 0]

    def pieces(self, rank: int):
        """(out_row, rows) of each launch (group) of rank's span, in launch
        order: the pieces a span travels in when it is sent launch by launch."""
        ls = self.launches[rank]
        return [(ls[g][3], sum((ls[g + i][2] - ls[g + i][1]) * self.band_h for i in range(n)))
                for g, n in self.groups[rank]]

    def recv_pieces(self):
        """(rank, row0, rows) of every launch's piece rank 0 receives, per rank
        in launch order (the order the pieces are sent in)."""
        return [(r, self.row0[r] + orow, n) for r in range(1, self.world) for orow, n in self.pieces(r) if n > 0]


class SpanTracer:
    """The launches of one rank's span of a batch (bench.py's trace for
    --partition spans; tests/test_gpu_dist.py replays them): launch j of
    plan.launches[rank] traces one frame's bands band_lo .. band_hi - 1
    (rt_render_batch_device with that band list; no list for a whole frame),
    packed at row out_row of the span buffer."""

    def __init__(self, ctx, width: int, height: int, max_bounces: int, plan: SpanPlan, rank: int = 0):
        self.ctx, self.W, self.H, self.B, self.plan, self.rank = ctx, width, height, max_bounces, plan, rank
        self.launches = plan.launches[rank]
        self.groups = plan.groups[rank]
        self._lists = [None if (lo, hi) == (0, plan.bpf) else np.arange(lo, hi, dtype=np.int32)
                       for (_, lo, hi, _) in self.launches]
        self._runs = [(np.ascontiguousarray([self.launches[g + i][1] for i in range(n)], dtype=np.int32),
                       np.ascontiguousarray([self.launches[g + i][2] for i in range(n)], dtype=np.int32))
                      for g, n in self.groups]

    def group_frames(self, j: int):
        """The frames (of the batch) of launch group j, in order."""
        g, n = self.groups[j]
        return [self.launches[g + i][0] for i in range(n)]

    def group_row(self, j: int) -> int:
        """The span buffer row where launch group j writes."""
        return self.launches[self.groups[j][0]][3]

    def launch_group(self, cams, j: int, stream: int, rgba_ptr, rad_ptr, stats=None) -> None:
        """Launch group j (cams: a ctypes array of its frames' CameraUBO) on
        `stream` into rgba_ptr / rad_ptr, the span buffer's row group_row(j)."""
        g, n = self.groups[j]
        if n == 1:
            return self.launch(cams[0], g, stream, rgba_ptr, rad_ptr, stats)
        lo, hi = self._runs[j]
        check(lib().rt_render_batch_runs_device(self.ctx, cams, n, self.W, self.H, self.B, self.plan.band_h,
                                                lo.ctypes.data_as(C.POINTER(C.c_int32)),
                                                hi.ctypes.data_as(C.POINTER(C.c_int32)), rgba_ptr, rad_ptr, stream,
                                                C.byref(stats) if stats is not None else None))

    def launch(self, cam, j: int, stream: int, rgba_ptr, rad_ptr, stats=None) -> None:
        """Launch j of the rank's span (cam: the CameraUBO of its frame) on
        `stream` into rgba_ptr / rad_ptr, the span buffer's row out_row
        (device pointers; rad_ptr may be None)."""
        L = lib()
        bl = self._lists[j]
        check(L.rt_render_batch_device(self.ctx, C.byref(cam), 1, self.W, self.H, self.B,
                                       self.plan.band_h if bl is not None else 0,
                                       bl.ctypes.data_as(C.POINTER(C.c_int32)) if bl is not None else None,
                                       len(bl) if bl is not None else 0, rgba_ptr, rad_ptr, stream,
                                       C.byref(stats) if stats is not None else None))


def _glob(group):
    import torch.distributed as dist
    return (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)


def _staged(group, t) -> bool:
    """gloo moves host memory only: device tensors are staged through the host."""
    import torch.distributed as dist
    return dist.get_backend(group) == "gloo" and t is not None and t.is_cuda


def wire_copy(rgba, rgb, pack: bool) -> None:
    """RGBA8 rows <-> RGB rows (the same [n, W, *] extent): on the device by
    rt_pack_rgb / rt_unpack_rgb (4 pixels a thread), else (host tensors, or
    rows not aligned for them) by a strided copy."""
    import torch
    n_px = rgba.shape[0] * rgba.shape[1]
    if (rgba.is_cuda and rgba.is_contiguous() and rgb.is_contiguous() and rgba.data_ptr() % 16 == 0
            and rgb.data_ptr() % 4 == 0):
        s = torch.cuda.current_stream(rgba.device).cuda_stream
        if pack:
            check(lib().rt_pack_rgb(rgba.data_ptr(), rgb.data_ptr(), n_px, s))
        else:
            check(lib().rt_unpack_rgb(rgb.data_ptr(), rgba.data_ptr(), n_px, s))
    elif pack:
        rgb.copy_(rgba[:, :, :3])
    else:
        rgba[:, :, :3].copy_(rgb)


def span_send(span, plan: SpanPlan, rgb=None, rad=None, group=None, rows=None) -> list:
    """Rank r > 0's send of its span of a batch: span is its [>= rows[r], W, 4]
    RGBA8 span buffer.  rgb (a [>= rows[r], W, 3] buffer): the rows travel as
    RGB, packed here (the alpha byte is always 255, compute_dynamic_ray.comp:235),
    3/4 of the bytes over the link.  rad: the span's float radiance, sent after.
    rows = (out_row, n): one launch's piece of the span only (plan.pieces; rank
    0 then posts span_post_recvs(..., pieces=True)).  One batch_isend_irecv
    (one RCCL group); returns its works (wait() orders the current stream after
    the send)."""
    import torch.distributed as dist
    rank = dist.get_rank(group)
    y, n = rows if rows is not None else (0, plan.rows[rank])
    if n == 0:
        return []
    src = span[y:y + n]
    if rgb is not None:
        wire_copy(src, rgb[y:y + n], pack=True)
        src = rgb[y:y + n]
    bufs = [src] + ([rad[y:y + n]] if rad is not None else [])
    ops = [dist.P2POp(dist.isend, b.cpu() if _staged(group, b) else b, _glob(group)(0), group) for b in bufs]
    return dist.batch_isend_irecv(ops)


def span_post_recvs(column, plan: SpanPlan, rgb=None, rad=None, group=None, pieces=False):
    """Rank 0's receives of every other span of a batch, posted at once:
    column is the batch's [n_frames * height, W, 4] RGBA8 frames (rank 0's
    own span traced in place), rgb (with the RGB wire) a [n_frames * height, W,
    3] landing the RGB rows arrive in, rad the batch's float radiance.
    pieces: one receive per launch of each span (the senders send launch by
    launch: span_send(rows=...)).  Returns (works, landings) for
    span_finish_recvs."""
    import torch
    import torch.distributed as dist
    glob = _glob(group)
    ops, landings = [], []
    for r, y0, n in (plan.recv_pieces() if pieces else plan.recv_slices()):
        for buf in ((rgb if rgb is not None else column),) + ((rad,) if rad is not None else ()):
            dst = buf[y0:y0 + n]
            if _staged(group, dst):
                landings.append((dst, torch.empty(dst.shape, dtype=dst.dtype)))
                dst = landings[-1][1]
            ops.append(dist.P2POp(dist.irecv, dst, glob(r), group))
    return (dist.batch_isend_irecv(ops) if ops else []), landings


def span_finish_recvs(works, landings, column, plan: SpanPlan, rgb=None) -> None:
    """Completes span_post_recvs: waits for the receives (NCCL: the current
    stream waits; gloo: the host), lands the host-staged rows, and with the RGB
    wire writes the received RGB rows into the RGBA8 frames (their alpha bytes
    must already be 255: set once when the frames buffer is made)."""
    for w in works:
        w.wait()
    for dst, host in landings:
        dst.copy_(host)
    sl = plan.recv_slices()
    if rgb is not None and sl:
        y = sl[0][1]                         # the received rows follow rank 0's span, to the column's end
        end = plan.n_frames * plan.height
        wire_copy(column[y:end], rgb[y:end], pack=False)


def exchange_spans(column, span, plan: SpanPlan, group=None, rgb=None, pieces=False) -> None:
    """One batch of the spans partition, both halves at once.  Rank 0: column
    is the batch's [n_frames * height, W, C] frames, its own span traced in
    place; every other span is received straight into its rows.  Rank r > 0:
    span is its [>= rows[r], W, C] span buffer, sent to rank 0.  rgb: the RGB
    wire (C = 4; span_send / span_post_recvs).  pieces: the spans travel launch
    by launch (bench.py's last batch of a phase).  On return the current
    stream is ordered after the exchange."""
    import torch.distributed as dist
    rank = dist.get_rank(group)
    if rank == 0:
        works, landings = span_post_recvs(column, plan, rgb=rgb, group=group, pieces=pieces)
        span_finish_recvs(works, landings, column, plan, rgb=rgb)
    else:
        for rows in (plan.pieces(rank) if pieces else [None]):
            for w in span_send(span, plan, rgb=rgb, group=group, rows=rows):
                w.wait()


# --- rotating row blocks (strong scaling, an option) -------------------------
#
# Each frame is cut into N contiguous row pieces, one per rank: rank 0's piece
# has h0 = root_share x H / N rows and the other N - 1 pieces split the rest
# evenly.  In frame k the pieces are laid out from row 0 in the rotated order
# k, k+1, ..., k-1 (mod N), so over any N consecutive frames every rank's
# piece visits N positions spread over the frame: the sky rows and the mesh
# rows are shared out while frames are in flight, as the interleaved bands
# share them within one frame.  What contiguity buys is the exchange: a
# rank's piece is one run of frame rows, so rank 0 receives it straight into
# the frame (RCCL point-to-point receives in one group, the gather's own
# primitive) and traces its own piece in place; there is no assembly pass.
# Rank 0 still does the most device work (its piece and every receive), so
# root_share < 1 gives it fewer rows (tools/rank0_exchange_bench.py,
# profiles/r02/rccl/).


def block_sizes(height: int, world: int, root_share: float = 1.0):
    """Rows of each rank's piece (rank 0 first)."""
    if world == 1:
        return [height]
    h0 = max(0, min(height, int(round(root_share * height / world))))
    rest = height - h0
    base, extra = divmod(rest, world - 1)
    return [h0] + [base + (1 if j < extra else 0) for j in range(world - 1)]


def block_layout(height: int, world: int, frame: int, root_share: float = 1.0):
    """Frame rows [y0, y1) of every rank's piece in frame `frame` (indexed by rank)."""
    sizes = block_sizes(height, world, root_share)
    out = [None] * world
    y = 0
    for j in range(world):
        r = (frame + j) % world
        out[r] = (y, y + sizes[r])
        y += sizes[r]
    return out


def exchange_blocks(frames, local, frame_ids, height: int, root_share: float = 1.0, group=None) -> None:
    """One batch of the blocks partition.  local[i]: this rank's piece of
    frame frame_ids[i] ([>= rows, W, C]).  frames[i] (rank 0 only): that
    frame's [height, W, C] buffer, whose own piece rank 0 has traced in place;
    every other rank's piece is received straight into its rows.  One
    batch_isend_irecv (one RCCL group of sends / receives); on return the
    current stream is ordered after it."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    # gloo moves host memory only: device tensors are staged through the host
    # (CPU tests and one-GPU rehearsals; RCCL sends and receives device memory)
    staged = dist.get_backend(group) == "gloo" and local is not None and local.is_cuda
    glob = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    ops, landings = [], []
    for i, f in enumerate(frame_ids):
        lay = block_layout(height, world, f, root_share)
        if rank == 0:
            for r in range(1, world):
                y0, y1 = lay[r]
                if y1 > y0:
                    dst = frames[i][y0:y1]
                    if staged:
                        landings.append((dst, dst.cpu()))
                        dst = landings[-1][1]
                    ops.append(dist.P2POp(dist.irecv, dst, glob(r), group))
        else:
            y0, y1 = lay[rank]
            if y1 > y0:
                src = local[i][: y1 - y0]
                ops.append(dist.P2POp(dist.isend, src.cpu() if staged else src, glob(0), group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for dst, host in landings:
        dst.copy_(host)


# --- frame batches (weak scaling) -------------------------------------------
#
# One frame tiled over N GPUs is bounded by its slowest wave (a few pixels'
# paths walk ~1,600 BVH nodes one dependent load after another),
# so it cannot scale strongly.  A batch of N frames of the render loop is tiled
# over the N GPUs instead: in frame f, rank r traces the bands b with
# b % N == (r + f) % N.  Over the batch every rank traces each band exactly
# once, so per-GPU work is one frame whatever N is; every frame is still split
# across all ranks and gathered to rank 0 over RCCL.


def batch_band_offset(frame: int, world: int, rank: int) -> int:
    """Band offset (rt_render_bands_device band_off) of rank in batch frame `frame`."""
    return (rank + frame) % world


class BatchPlan:
    """Row bookkeeping of an n_frames batch over world ranks (band_h-row bands)."""

    def __init__(self, height: int, band_h: int, world: int, n_frames: int, rotate: bool = True):
        # rotate: frame f of the batch gives rank r the bands (r + f) mod world
        # (frames partition); else every frame gives rank r the bands r (a
        # batch of consecutive one-frame steps of the bands partition)
        self.height, self.band_h, self.world, self.n_frames = height, band_h, world, n_frames
        self.rows = [[band_rows(height, band_h, world, batch_band_offset(f, world, r) if rotate else r)
                      for f in range(n_frames)] for r in range(world)]
        self.max_rows = max(len(x) for per_rank in self.rows for x in per_rank)
        # source row (in the gathered [world, n_frames, max_rows] stack) of every
        # row of every frame: one index_select assembles the whole batch
        src = np.empty(n_frames * height, np.int64)
        for r in range(world):
            for f in range(n_frames):
                rows = self.rows[r][f]
                src[f * height + rows] = (r * n_frames + f) * self.max_rows + np.arange(len(rows))
        self.src = src

    def local_rows(self, rank: int, frame: int) -> int:
        return len(self.rows[rank][frame])


_PLANS: dict = {}


def _cached_plan(height: int, band_h: int, world: int, n_frames: int, device, rotate: bool = True):
    """BatchPlan and its source-row index on `device`, built once per layout."""
    import torch
    key = (height, band_h, world, n_frames, str(device), rotate)
    hit = _PLANS.get(key)
    if hit is None:
        plan = BatchPlan(height, band_h, world, n_frames, rotate)
        hit = (plan, torch.as_tensor(plan.src, device=device))
        _PLANS[key] = hit
    return hit


def gather_batch(local, plan: BatchPlan, group=None, src_index=None):
    """local: this rank's [n_frames, max_rows, W, C] packed bands (torch).
    Returns the [n_frames, height, W, C] frames on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    stack = gl = None
    if rank == 0:                  # gather straight into one [world, ...] tensor (views, no extra copy)
        stack = torch.empty((plan.world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
        gl = list(stack.unbind(0))
    dist.gather(local, gl, dst=0, group=group)
    if rank != 0:
        return None
    stack = stack.reshape(plan.world * plan.n_frames * plan.max_rows, -1)
    if src_index is None:
        src_index = torch.as_tensor(plan.src, device=local.device)
    out = torch.index_select(stack, 0, src_index)
    return out.reshape((plan.n_frames, plan.height) + tuple(local.shape[2:]))


class DistRenderer:
    """Renders frames over all ranks: each rank traces its bands on its GPU
    with rt_render_bands_device, then gather_frame assembles rank 0's copy."""

    def __init__(self, renderer, band_h: int = 16, group=None):
        import torch
        import torch.distributed as dist
        self.r = renderer
        self.band_h = band_h
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = torch.device("cuda", torch.cuda.current_device())

    def trace_local(self, camera, width: int, height: int, max_bounces: int, out=None, stream=None):
        import torch
        from .engine import _ubo
        rows = band_row_count(height, self.band_h, self.world, self.rank)
        if out is None:
            out = torch.empty((rows, width, 4), dtype=torch.uint8, device=self.device)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        check(lib().rt_render_bands_device(self.r._ctx, C.byref(_ubo(camera)), width, height, max_bounces,
                                           self.band_h, self.world, self.rank, out.data_ptr(), None,
                                           s.cuda_stream, None))
        return out

    def render(self, camera, width: int, height: int, max_bounces: int):
        local = self.trace_local(camera, width, height, max_bounces)
        return gather_frame(local, height, self.band_h, self.group)
