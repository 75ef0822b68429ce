// rt_wire.hip — the multi-GPU wire format of the frames (rtamd/dist.py
// span_send / span_finish_recvs).
//
// The reference's RGBA8 frame always has alpha 255 (imageStore of
// vec4(color, 1.0), compute_dynamic_ray.comp:235), so a rank's rows cross the
// xGMI link as RGB: 3 of the 4 bytes.  rt_pack_rgb packs RGBA8 pixels to RGB
// before a send; rt_unpack_rgb writes received RGB pixels back as RGBA8 with
// alpha 255.  Both move 4 pixels per thread (one 16-B RGBA load or store, three
// 4-B RGB words), so they run at copy speed; a strided torch copy of the same
// bytes cost the sending rank 15% of its frame time (profiles/r05/r5ao).
#include "rt_internal.h"

namespace rtamd {
namespace {

__global__ __launch_bounds__(256) void pack_rgb(const uint4* __restrict__ rgba, uint32_t* __restrict__ rgb,
                                                size_t groups) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= groups) return;
    const uint4 p = rgba[g];                         // 4 pixels, R | G << 8 | B << 16 | A << 24 each
    const uint32_t a = p.x & 0xFFFFFFu, b = p.y & 0xFFFFFFu, c = p.z & 0xFFFFFFu, d = p.w & 0xFFFFFFu;
    rgb[3 * g + 0] = a | (b << 24);
    rgb[3 * g + 1] = (b >> 8) | (c << 16);
    rgb[3 * g + 2] = (c >> 16) | (d << 8);
}

__global__ __launch_bounds__(256) void unpack_rgb(const uint32_t* __restrict__ rgb, uint4* __restrict__ rgba,
                                                  size_t groups) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= groups) return;
    const uint32_t w0 = rgb[3 * g + 0], w1 = rgb[3 * g + 1], w2 = rgb[3 * g + 2];
    uint4 p;
    p.x = (w0 & 0xFFFFFFu) | 0xFF000000u;
    p.y = ((w0 >> 24) | (w1 << 8)) | 0xFF000000u;
    p.z = ((w1 >> 16) | (w2 << 16)) | 0xFF000000u;
    p.w = (w2 >> 8) | 0xFF000000u;
    rgba[g] = p;
}

// the last n % 4 pixels, one per thread
__global__ void pack_tail(const uint8_t* __restrict__ rgba, uint8_t* __restrict__ rgb, size_t n) {
    const size_t i = threadIdx.x;
    if (i >= n) return;
    for (int c = 0; c < 3; ++c) rgb[3 * i + c] = rgba[4 * i + c];
}

__global__ void unpack_tail(const uint8_t* __restrict__ rgb, uint8_t* __restrict__ rgba, size_t n) {
    const size_t i = threadIdx.x;
    if (i >= n) return;
    for (int c = 0; c < 3; ++c) rgba[4 * i + c] = rgb[3 * i + c];
    rgba[4 * i + 3] = 255;
}

}  // namespace

hipError_t wire_pack(const void* rgba, void* rgb, size_t n_px, hipStream_t s) {
    const size_t groups = n_px / 4, rest = n_px % 4;
    if (groups) {
        hipLaunchKernelGGL(pack_rgb, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s,
                           static_cast<const uint4*>(rgba), static_cast<uint32_t*>(rgb), groups);
    }
    if (rest) {
        hipLaunchKernelGGL(pack_tail, dim3(1), dim3(4), 0, s, static_cast<const uint8_t*>(rgba) + 16 * groups,
                           static_cast<uint8_t*>(rgb) + 12 * groups, rest);
    }
    return hipGetLastError();
}

hipError_t wire_unpack(const void* rgb, void* rgba, size_t n_px, hipStream_t s) {
    const size_t groups = n_px / 4, rest = n_px % 4;
    if (groups) {
        hipLaunchKernelGGL(unpack_rgb, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s,
                           static_cast<const uint32_t*>(rgb), static_cast<uint4*>(rgba), groups);
    }
    if (rest) {
        hipLaunchKernelGGL(unpack_tail, dim3(1), dim3(4), 0, s, static_cast<const uint8_t*>(rgb) + 12 * groups,
                           static_cast<uint8_t*>(rgba) + 16 * groups, rest);
    }
    return hipGetLastError();
}

}  // namespace rtamd
