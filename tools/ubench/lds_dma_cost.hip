// lds_dma_cost.hip — microbenchmark (analysis aid, not part of the product):
// what a wave-uniform BVH step's record fetch costs the vector memory
// pipeline on gfx950, by instruction form.  ta_cost.hip measured a
// global_load_dwordx4 at ~17 cycles per wave instruction per CU whatever
// the active lanes when every lane reads one address, and a 4-byte load at
// ~6.  The walk's uniform step needs a 32-byte node record in every lane.
// Forms, each `iters` rounds of 8 independent fetches of a 32-B record
// (addresses do not depend on loaded data), all hitting L1/L2:
//   0: two global_load_dwordx4, every lane the same address (walk 2 today)
//   1: one global_load_dwordx4 on 2 lanes (16 B each) -> LDS (ds_write_b128)
//      -> two ds_read_b128 by every lane (walk 12's staging)
//   2: one global_load_lds_dwordx4 on 2 lanes (LDS-DMA) -> two ds_read_b128
//   3: one global_load_dword on 8 lanes (4 B each) -> LDS (ds_write_b32)
//      -> two ds_read_b128
//   4: one global_load_lds_dword on 8 lanes -> two ds_read_b128
// Prints ns and cycles per record fetch per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int kTable = 16384;   // float4 entries: 256 KB

template <int MODE>
__global__ __launch_bounds__(64) void fetch(const float4* __restrict__ t, float* out, int iters) {
    __shared__ float4 stage[8][2];
    const int lane = threadIdx.x;
    float acc = 0.f;
    unsigned base = (blockIdx.x * 977u) & (kTable - 1);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            unsigned j = (base + (unsigned)(i * 8 + k) * 67u) & (kTable - 2);   // a 32-B record
            // in a VGPR, as a walk's per-lane node index is: the compiler must
            // not turn a provably uniform address into scalar loads
            asm volatile("" : "+v"(j));
            if (MODE == 0) {
                const float4 a = t[j], b = t[j + 1];
                acc += ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
            } else if (MODE == 1) {
                if (lane < 2) stage[k][lane] = t[j + lane];
            } else if (MODE == 2) {
                if (lane < 2)
                    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(t + j + lane),
                                                     (__attribute__((address_space(3))) void*)(
                                                         &stage[k][0]), 16, 0, 0);
            } else if (MODE == 3) {
                if (lane < 8) reinterpret_cast<float*>(&stage[k][0])[lane] = reinterpret_cast<const float*>(t + j)[lane];
            } else {
                if (lane < 8)
                    __builtin_amdgcn_global_load_lds(reinterpret_cast<const float*>(t + j) + lane,
                                                     (__attribute__((address_space(3))) void*)(
                                                         &stage[k][0]), 4, 0, 0);
            }
        }
        if (MODE != 0) {
            __builtin_amdgcn_s_waitcnt(0);   // vmcnt/lgkmcnt 0: the staged records have landed
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float4 a = stage[k][0], b = stage[k][1];
                acc += ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
            }
            __syncthreads();
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
    const char* names[] = {"2x global_load_dwordx4, all lanes one address",
                           "global_load_dwordx4 on 2 lanes -> ds_write -> 2x ds_read_b128",
                           "global_load_lds_dwordx4 on 2 lanes -> 2x ds_read_b128",
                           "global_load_dword on 8 lanes -> ds_write -> 2x ds_read_b128",
                           "global_load_lds_dword on 8 lanes -> 2x ds_read_b128"};
    for (int blocks_per_cu : {16, 32}) {
        const int blocks = n_cu * blocks_per_cu;
        for (int mode = 0; mode < 5; ++mode) {
            auto k = mode == 0 ? fetch<0> : mode == 1 ? fetch<1> : mode == 2 ? fetch<2> : mode == 3 ? fetch<3> : fetch<4>;
            hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, t, out, 4);
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, t, out, iters);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0.f;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double per_cu = (double)blocks / n_cu * iters * 8;   // record fetches per CU
            std::printf("waves/CU %2d  mode %d  %-64s %.3f ms  %.2f ns/fetch/CU  %.1f cyc@2.4GHz\n", blocks_per_cu,
                        mode, names[mode], ms, ms * 1e6 / per_cu, ms * 1e6 / per_cu * 2.4);
        }
    }
    return 0;
}
