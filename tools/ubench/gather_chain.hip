// gather_chain.hip — microbenchmark (analysis aid): latency of one wave's
// dependent load chain on gfx950, for coherent vs lane-divergent addresses and
// for 1, 2 or 5 16-B loads per lane per step (the walk's node / node+leaf
// records).  Prints ns per step.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/gather_chain.hip -o /tmp/gather_chain
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

template <int LOADS>
__global__ void chain(const float4* __restrict__ t, unsigned n_rec, int steps, int divergent, unsigned long long* out,
                      float* sink) {
    const int lane = threadIdx.x & 63;
    unsigned i = divergent ? (lane * 2654435761u) % n_rec : 12345u % n_rec;
    float acc = 0.f;
    __syncthreads();
    const unsigned long long t0 = wall_clock64();
    for (int s = 0; s < steps; ++s) {
        const float4* r = t + (size_t)i * 8;     // 128-B records
        float4 q[LOADS];
#pragma unroll
        for (int k = 0; k < LOADS; ++k) q[k] = r[k];
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < LOADS; ++k) v += q[k].x + q[k].w;
        acc += v;
        i = (__float_as_uint(q[0].y) + (divergent ? 0u : 0u)) % n_rec;   // next record comes from the data
    }
    const unsigned long long t1 = wall_clock64();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    sink[threadIdx.x] = acc;
}

int main() {
    int dev_clock_khz = 0;
    hipDeviceGetAttribute(&dev_clock_khz, hipDeviceAttributeWallClockRate, 0);
    for (size_t mb : {2, 8, 64}) {
        const unsigned n_rec = (unsigned)(mb * 1024 * 1024 / 128);
        std::vector<float> h((size_t)n_rec * 32);
        srand(1);
        for (size_t r = 0; r < n_rec; ++r) {
            unsigned nxt = (unsigned)(((unsigned long long)rand() * 2654435761ull + r) % n_rec);
            for (int k = 0; k < 32; ++k) h[r * 32 + k] = 1.0f;
            unsigned u = nxt;
            memcpy(&h[r * 32 + 1], &u, 4);   // q[0].y holds the next record
        }
        float4* d;
        float* sink;
        unsigned long long* o;
        hipMalloc(&d, h.size() * 4);
        hipMalloc(&sink, 1024 * 4);
        hipMalloc(&o, 8);
        hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
        const int steps = 2000;
        for (int div = 0; div < 2; ++div)
            for (int loads : {1, 2, 5}) {
                unsigned long long ticks = 0;
                for (int rep = 0; rep < 3; ++rep) {
                    if (loads == 1) hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, d, n_rec, steps, div, o, sink);
                    if (loads == 2) hipLaunchKernelGGL(chain<2>, dim3(1), dim3(64), 0, 0, d, n_rec, steps, div, o, sink);
                    if (loads == 5) hipLaunchKernelGGL(chain<5>, dim3(1), dim3(64), 0, 0, d, n_rec, steps, div, o, sink);
                    hipDeviceSynchronize();
                    hipMemcpy(&ticks, o, 8, hipMemcpyDeviceToHost);
                }
                const double ns = ticks * 1e6 / dev_clock_khz / steps;
                printf("table %3zu MB  %s  %d x 16 B per lane per step: %.0f ns per step\n", mb,
                       div ? "divergent (64 lines)" : "coherent  (1 line)  ", loads, ns);
            }
        hipFree(d);
        hipFree(sink);
        hipFree(o);
    }
    return 0;
}
