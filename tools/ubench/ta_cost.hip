// ta_cost.hip — microbenchmark (analysis aid, not part of the product): the
// cost of vector memory loads on gfx950 as a function of active lanes, load
// width and address pattern, all hitting L1/L2 (a 256 KB table).
//
// Every wave runs `iters` rounds of 8 independent loads (addresses do not
// depend on loaded data), so the kernel is bound by the load pipeline
// (texture addresser / data return), not by latency.  Prints one line per
// variant: ns per wave-load instruction per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int kTable = 16384;   // float4 entries: 256 KB

// mode m >= 0: lane byte stride 16 << m ... as float4 index stride 1 << m
//   (m = 0: consecutive 16-B entries; 1: 32 B; 2: 64 B; 3: 128 B; 4: 256 B)
// mode -1: every lane the same entry
template <int WIDTH>
__global__ __launch_bounds__(64) void loads(const float4* __restrict__ t, float* out, int iters, int active, int mode) {
    const int lane = threadIdx.x;
    float acc = 0.f;
    if (lane < active) {
        unsigned base = (blockIdx.x * 977u) & (kTable - 1);
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                unsigned j = base + (unsigned)(i * 8 + k) * 67u;
                j = mode < 0 ? j : j + ((unsigned)lane << mode);
                j &= kTable - 1;
                if (WIDTH == 16) {
                    const float4 v = t[j];
                    acc += (v.x + v.y) + (v.z + v.w);
                } else if (WIDTH == 8) {
                    const float2 v = reinterpret_cast<const float2*>(t)[2 * j];
                    acc += v.x + v.y;
                } else {
                    acc += reinterpret_cast<const float*>(t)[4 * j];
                }
            }
        }
    }
    if (acc == 12345.f) out[0] = acc;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 256;
    int dev = 0, n_cu = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    float4* t = nullptr;
    float* out = nullptr;
    CHECK(hipMalloc(&t, kTable * sizeof(float4)));
    CHECK(hipMalloc(&out, 64));
    std::vector<float4> h(kTable);
    for (int i = 0; i < kTable; ++i) h[i] = make_float4((float)i, 1.f, 2.f, 3.f);
    CHECK(hipMemcpy(t, h.data(), kTable * sizeof(float4), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int blocks = n_cu * 16;   // 16 one-wave workgroups per CU
    for (int width : {16, 8, 4}) {
        for (int mode : {-1, 0, 1, 2, 3, 4}) {
            for (int active : {64, 16}) {
                auto k = width == 16 ? loads<16> : width == 8 ? loads<8> : loads<4>;
                hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, t, out, 4, active, mode);
                CHECK(hipEventRecord(e0));
                hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, t, out, iters, active, mode);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms = 0.f;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                const double per_cu = (double)blocks / n_cu * iters * 8;   // wave-load instructions per CU
                std::printf("width %2d B  stride %3d B  active %2d  %.3f ms  %.2f ns/wave-load/CU  %.1f cyc@2.4GHz\n",
                            width, mode < 0 ? 0 : 16 << mode, active, ms, ms * 1e6 / per_cu, ms * 1e6 / per_cu * 2.4);
            }
        }
    }
    return 0;
}
