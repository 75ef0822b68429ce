// rt_learn.hip — the heavy-first order learned on the device (option
// heavy_first, rt_runtime.hip plan_order).
//
// A learning launch (the diagnostic build of trace_simple) leaves, per tile,
// its wave's duration and lockstep steps (diag words 0-1, 4-5) and, per pixel,
// its walk length (diag_lane).  The host used to copy those back (8 MB of
// per-pixel lengths for a 1080p frame), sort the tiles and pick the heavy
// pixels, behind a stream synchronisation: the first frame after the camera
// stops cost 4.4 ms (profiles/r03/evidence_r3fin2/bench_orbit.json).  Here the
// same order is computed by a few small kernels on the stream that ran the
// learning launch, and only the heavy-pixel count comes back (4 bytes, read by
// the host once an event says it is there), so no launch ever waits:
//
//   learn_costs    tile k's cost (duration, or steps + 2 x windows), the
//                  total lockstep steps and the costliest tile
//   learn_split    option order_split: tiles below p% of the costliest keep
//                  their raster order (cost key 0)
//   radix sort     tiles by cost, descending and stable (rocPRIM), so equal
//                  keys keep raster order, as the host's stable_sort did
//   learn_cand     every pixel's key: its walk length and pixel index if the
//                  length exceeds the heavy-pixel bar (the bulk estimate: total
//                  steps x concurrent launches / resident waves x
//                  heavy_pixel_factor), else 0
//   radix sort     the keys, descending (rocPRIM): length first, then the
//                  lower pixel index, a total order, so the choice is the
//                  host's whatever the candidate count
//   learn_top      the first `cap` non-zero keys become the heavy pixels and
//                  their tiles' lane masks
//
// The order only decides which wave traces a pixel and when, never what it
// computes, so results are identical whatever these kernels choose.
#include <rocprim/device/device_radix_sort.hpp>

#include "rt_internal.h"

namespace rtamd {

struct LearnScratch {
    unsigned long long total;    // sum of the tiles' lockstep steps + 2 x windows
    unsigned long long cmax;     // the costliest tile's cost
    unsigned ncand;              // unused (round 5: every pixel has a key)
    unsigned pad[3];
};

namespace {

constexpr size_t kAlign = 256;

size_t up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

struct Layout {
    size_t hdr, key_in, key_out, val_in, cand, cand_out, temp, temp_bytes, total;
};

Layout layout(int n) {
    Layout L{};
    size_t off = 0;
    L.hdr = off;     off += up(sizeof(LearnScratch));
    L.key_in = off;  off += up(sizeof(unsigned) * (size_t)n);
    L.key_out = off; off += up(sizeof(unsigned) * (size_t)n);
    L.val_in = off;  off += up(sizeof(int) * (size_t)n);
    const size_t nl = (size_t)n * 64;
    L.cand = off;    off += up(sizeof(unsigned long long) * nl);
    L.cand_out = off; off += up(sizeof(unsigned long long) * nl);
    L.temp = off;
    size_t tb = 0, tc = 0;
    (void)rocprim::radix_sort_pairs_desc(nullptr, tb, (const unsigned*)nullptr, (unsigned*)nullptr,
                                         (const int*)nullptr, (int*)nullptr, n, 0, 32);
    (void)rocprim::radix_sort_keys_desc(nullptr, tc, (const unsigned long long*)nullptr,
                                        (unsigned long long*)nullptr, nl, 0, 64);
    size_t tx = 0;
    (void)rocprim::radix_sort_pairs(nullptr, tx, (const unsigned*)nullptr, (unsigned*)nullptr,
                                    (const int*)nullptr, (int*)nullptr, n, 0, 3);
    tb = tb > tx ? tb : tx;
    L.temp_bytes = up(tb > tc ? tb : tc);
    off += L.temp_bytes;
    L.total = off;
    return L;
}

__global__ __launch_bounds__(256) void learn_costs(const unsigned long long* __restrict__ rec, int off, int n,
                                                   int learn_cost, unsigned* __restrict__ key,
                                                   int* __restrict__ val, LearnScratch* hdr) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long steps = 0, cost = 0;
    if (k < n) {
        const unsigned long long* r = rec + 8 * ((size_t)off + (size_t)k);
        steps = r[4] + 2 * r[5];
        cost = learn_cost == 0 ? steps : r[1] - r[0];
        key[k] = (unsigned)(cost < 0xFFFFFFFFull ? cost : 0xFFFFFFFFull);
        val[k] = k;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        steps += __shfl_xor(steps, o);
        const unsigned long long c2 = __shfl_xor(cost, o);
        cost = c2 > cost ? c2 : cost;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&hdr->total, steps);
        atomicMax(&hdr->cmax, cost);
    }
}

// order_split: a tile whose cost is below pct% of the costliest keeps its
// raster place (key 0; the stable sort leaves such tiles in index order).
__global__ __launch_bounds__(256) void learn_split(unsigned* __restrict__ key, int n, const LearnScratch* hdr,
                                                   int pct) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double split_at = (double)pct / 100.0 * (double)hdr->cmax;
    if (!((double)key[k] >= split_at)) key[k] = 0u;
}

// A candidate's sort key: walk length high, then the complement of its pixel
// index, so a descending sort puts longer walks first and, among equal ones,
// the lower pixel index first (the host's stable_sort order).
__global__ __launch_bounds__(256) void learn_cand(const unsigned* __restrict__ lane, size_t nl,
                                                  const LearnScratch* hdr, double bar_scale,
                                                  unsigned long long* __restrict__ cand) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nl) return;
    const unsigned len = lane[q];
    const double bar = bar_scale * (double)hdr->total;
    cand[q] = (double)len > bar ? ((unsigned long long)len << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)q)
                                : 0ull;
}

// sorted: every pixel's key, descending; the first cap non-zero ones are the
// heavy pixels (a non-zero key's length is >= 1, so it sorts above every 0).
__global__ __launch_bounds__(256) void learn_top(const unsigned long long* __restrict__ sorted, int cap,
                                                 int* __restrict__ hpix, unsigned long long* __restrict__ mask,
                                                 int* __restrict__ nhpix) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap) return;
    const unsigned long long k = sorted[i];
    if (i == 0 && k == 0ull) *nhpix = 0;
    if (k == 0ull) return;
    const int q = (int)(0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFull));
    hpix[i] = q;
    atomicOr(&mask[q >> 6], 1ull << (q & 63));
    if (i + 1 == cap || sorted[i + 1] == 0ull) *nhpix = i + 1;      // the last heavy pixel
}

// Option xcd_order: the eighth of the tiles (0-7) sorted position i's tile
// belongs to, by its rank in the order (row class, row, frame, column), a
// row's class being (row / band) % 8: XCD c's tiles are then rows of one class
// (a band of rows every 8 bands), so its L2 serves rays from fewer parts of
// the scene.
__global__ __launch_bounds__(256) void xcd_keys(const int* __restrict__ order, int n, int tiles_x, int tiles_y,
                                                int frames, int band, unsigned* __restrict__ key,
                                                int* __restrict__ val) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int t = order[i];
    const int col = t % tiles_x, by = t / tiles_x;
    const int f = by / tiles_y, row = by - f * tiles_y;
    // rows of each class: full cycles of 8 bands, then the last partial cycle
    const int cyc = 8 * band, full = tiles_y / cyc, rem = tiles_y - full * cyc;
    const int c = (row / band) % 8;
    int before = 0;                                      // rows of the classes below c
    for (int q = 0; q < c; ++q) before += full * band + min(max(rem - q * band, 0), band);
    const int prow = before + (row / cyc) * band + row % band;   // the row's place in class order
    const long long rank = ((long long)prow * frames + f) * tiles_x + col;
    key[i] = (unsigned)(rank / (n / 8));
    val[i] = t;
}

// sorted: the tiles grouped by eighth (stable: most expensive first within
// each); position r * 8 + c takes eighth c's r-th tile.
__global__ __launch_bounds__(256) void xcd_place(const int* __restrict__ sorted, int n, int* __restrict__ order) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int m = n / 8, c = j / m, r = j - c * m;
    order[r * 8 + c] = sorted[j];
}

}  // namespace

size_t learn_scratch_bytes(int n) { return layout(n).total; }

hipError_t learn_on_device(const LearnParams& lp, const unsigned long long* rec, const unsigned* lane,
                           void* scratch, int* d_order, unsigned long long* d_mask, int* d_hpix, int* d_nhpix,
                           hipStream_t s) {
    const Layout L = layout(lp.n);
    char* base = static_cast<char*>(scratch);
    LearnScratch* hdr = reinterpret_cast<LearnScratch*>(base + L.hdr);
    unsigned* key_in = reinterpret_cast<unsigned*>(base + L.key_in);
    unsigned* key_out = reinterpret_cast<unsigned*>(base + L.key_out);
    int* val_in = reinterpret_cast<int*>(base + L.val_in);
    unsigned long long* cand = reinterpret_cast<unsigned long long*>(base + L.cand);
    hipError_t e = hipMemsetAsync(hdr, 0, sizeof(LearnScratch), s);
    if (e == hipSuccess) e = hipMemsetAsync(d_mask, 0, sizeof(unsigned long long) * (size_t)lp.n, s);
    if (e != hipSuccess) return e;
    const int g = (lp.n + 255) / 256;
    hipLaunchKernelGGL(learn_costs, dim3(g), dim3(256), 0, s, rec, lp.rec_off, lp.n, lp.learn_cost, key_in, val_in,
                       hdr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (lp.order_split > 0) {
        hipLaunchKernelGGL(learn_split, dim3(g), dim3(256), 0, s, key_in, lp.n, hdr, lp.order_split);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    size_t tb = L.temp_bytes;
    e = rocprim::radix_sort_pairs_desc(base + L.temp, tb, key_in, key_out, val_in, d_order, lp.n, 0, 32, s);
    if (e != hipSuccess) return e;
    if (lp.xcd > 0 && lp.n % 8 == 0 && lp.tiles_x > 0 && lp.tiles_y > 0 && lp.frames > 0 &&
        (long long)lp.tiles_x * lp.tiles_y * lp.frames == lp.n) {
        int* sorted = reinterpret_cast<int*>(base + L.cand);            // free until learn_cand
        hipLaunchKernelGGL(xcd_keys, dim3(g), dim3(256), 0, s, d_order, lp.n, lp.tiles_x, lp.tiles_y, lp.frames,
                           lp.xcd, key_in, val_in);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        tb = L.temp_bytes;
        e = rocprim::radix_sort_pairs(base + L.temp, tb, key_in, key_out, val_in, sorted, lp.n, 0, 3, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(xcd_place, dim3(g), dim3(256), 0, s, sorted, lp.n, d_order);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const size_t nl = (size_t)lp.n * 64;
    unsigned long long* cand_out = reinterpret_cast<unsigned long long*>(base + L.cand_out);
    hipLaunchKernelGGL(learn_cand, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, s, lane, nl, hdr,
                       lp.bar_scale, cand);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tb = L.temp_bytes;
    e = rocprim::radix_sort_keys_desc(base + L.temp, tb, cand, cand_out, nl, 0, 64, s);
    if (e != hipSuccess) return e;
    const int cap = (int)std::min<size_t>((size_t)std::max(lp.cap, 0), nl);
    if (cap == 0) return hipMemsetAsync(d_nhpix, 0, sizeof(int), s);
    hipLaunchKernelGGL(learn_top, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, s, cand_out, cap, d_hpix,
                       d_mask, d_nhpix);
    return hipGetLastError();
}

}  // namespace rtamd
