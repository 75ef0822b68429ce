/* layout_sim.c — L2 model of one XCD for tools/layout_model.py (analysis aid,
 * not part of the product).
 *
 * Input: the lockstep steps of a sequence of tile waves (CSR: tile -> steps,
 * step -> the distinct nodes its walking lanes visit) and a storage layout
 * (node -> up to 3 128-B line numbers, -1 = none).  `resident` waves run at
 * once, one step each per round, a finished wave's slot taking the next tile
 * (dispatch order = input order).  Each step's lines go through a
 * set-associative LRU cache (sets x ways); the result is the count of line
 * accesses and of misses (what the L2 fetches).
 *
 * Build: gcc -O2 -shared -fPIC -o tools/liblayout_sim.so tools/layout_sim.c
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int64_t* tag;
    uint32_t* age;
    int sets, ways;
    uint32_t clock;
} cache_t;

static int cache_access(cache_t* c, int64_t line) {
    const int s = (int)((uint64_t)(line * 0x9E3779B97F4A7C15ull) >> 40) % c->sets;
    int64_t* t = c->tag + (size_t)s * c->ways;
    uint32_t* a = c->age + (size_t)s * c->ways;
    int victim = 0;
    ++c->clock;
    for (int w = 0; w < c->ways; ++w) {
        if (t[w] == line) { a[w] = c->clock; return 1; }
        if (a[w] < a[victim]) victim = w;
    }
    t[victim] = line;
    a[victim] = c->clock;
    return 0;
}

/* A negative node entry -(x + 1) is a cooperative-tail window starting at
 * node x: every node whose walk slot lies in [slot(x), slot(x) + window) is
 * loaded (node_slot: the walk-slot number the window counts in). */
int64_t layout_sim(int n_tiles, const int64_t* tile_ptr, const int64_t* step_ptr, const int32_t* nodes,
                   const int64_t* node_lines, const int64_t* node_slot, int64_t n_nodes, int window,
                   int resident, int sets, int ways, int64_t* out_accesses) {
    cache_t c;
    c.sets = sets;
    c.ways = ways;
    c.clock = 0;
    c.tag = malloc(sizeof(int64_t) * (size_t)sets * ways);
    c.age = calloc((size_t)sets * ways, sizeof(uint32_t));
    for (size_t i = 0; i < (size_t)sets * ways; ++i) c.tag[i] = -1;
    int64_t* cur = malloc(sizeof(int64_t) * (size_t)resident);   /* a slot's next step */
    int64_t* end = malloc(sizeof(int64_t) * (size_t)resident);
    int next_tile = 0, live = 0;
    for (int r = 0; r < resident; ++r) {
        cur[r] = end[r] = 0;
        while (next_tile < n_tiles && tile_ptr[next_tile] == tile_ptr[next_tile + 1]) ++next_tile;
        if (next_tile < n_tiles) {
            cur[r] = tile_ptr[next_tile];
            end[r] = tile_ptr[next_tile + 1];
            ++next_tile;
            ++live;
        }
    }
    int64_t acc = 0, miss = 0;
    enum { kSeen = 512 };
    int64_t seen[kSeen];
    while (live > 0) {
        for (int r = 0; r < resident; ++r) {
            if (cur[r] >= end[r]) continue;
            const int64_t st = cur[r]++;
            int ns = 0;
            for (int64_t k = step_ptr[st]; k < step_ptr[st + 1]; ++k) {
                int64_t x = nodes[k], last = x;
                if (x < 0) {                                  /* a window */
                    x = -x - 1;
                    last = x;
                    while (last + 1 < n_nodes && node_slot[last + 1] < node_slot[x] + window) ++last;
                }
                for (int64_t y = x; y <= last; ++y) {
                    const int64_t* nl = node_lines + 3 * (size_t)y;
                    for (int j = 0; j < 3 && nl[j] >= 0; ++j) {
                        int dup = 0;
                        for (int q = ns - 1; q >= 0 && q >= ns - 8; --q) if (seen[q] == nl[j]) { dup = 1; break; }
                        if (!dup) for (int q = 0; q < ns - 8; ++q) if (seen[q] == nl[j]) { dup = 1; break; }
                        if (!dup && ns < kSeen) seen[ns++] = nl[j];
                    }
                }
            }
            for (int q = 0; q < ns; ++q) {
                ++acc;
                if (!cache_access(&c, seen[q])) ++miss;
            }
            if (cur[r] >= end[r]) {
                --live;
                while (next_tile < n_tiles && tile_ptr[next_tile] == tile_ptr[next_tile + 1]) ++next_tile;
                if (next_tile < n_tiles) {
                    cur[r] = tile_ptr[next_tile];
                    end[r] = tile_ptr[next_tile + 1];
                    ++next_tile;
                    ++live;
                }
            }
        }
    }
    free(c.tag);
    free(c.age);
    free(cur);
    free(end);
    *out_accesses = acc;
    return miss;
}
