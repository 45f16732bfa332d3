// vx_synth.hip — device generator for synthetic piece batches (bench/test
// plumbing, not the hashing path).  Device twin of oracle/sha1_oracle.c
// vxo_gen_piece; spec in DESIGN.md "Synthetic pieces":
//   key  = mix64(seed ^ (p * 0xD1B54A32D192ED03))
//   w[i] = mix64(key + (i + 1) * 0x9E3779B97F4A7C15)   (little-endian bytes)
//   corrupt: p % ce == ce-1  ->  byte (p * 7919) % len ^= 0xFF
// The CPU can therefore regenerate any piece of a 16 GiB device batch to
// check its digest.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vx_kernels.h"

namespace vx {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void synth_fill_kernel(uint8_t* __restrict__ base, uint64_t stride, uint32_t len,
                                                         uint32_t n, uint64_t first, uint64_t seed) {
    const uint32_t chunks = (len + 15) / 16;  // 16-byte chunks per piece
    const uint64_t total = (uint64_t)chunks * n;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = (uint32_t)(t / chunks);
        const uint32_t c = (uint32_t)(t - (uint64_t)p * chunks);
        const uint64_t key = mix64(seed ^ ((first + p) * 0xD1B54A32D192ED03ULL));
        const uint64_t w0 = mix64(key + (uint64_t)(2 * c + 1) * 0x9E3779B97F4A7C15ULL);
        const uint64_t w1 = mix64(key + (uint64_t)(2 * c + 2) * 0x9E3779B97F4A7C15ULL);
        uint8_t* dst = base + (uint64_t)p * stride + 16ull * c;
        if (16u * c + 16u <= len) {
            uint4 v;
            v.x = (uint32_t)w0;
            v.y = (uint32_t)(w0 >> 32);
            v.z = (uint32_t)w1;
            v.w = (uint32_t)(w1 >> 32);
            *reinterpret_cast<uint4*>(dst) = v;
        } else {
            const uint32_t nb = len - 16u * c;
            for (uint32_t b = 0; b < nb; ++b) dst[b] = (uint8_t)((b < 8 ? w0 >> (8 * b) : w1 >> (8 * (b - 8))));
        }
    }
}

__global__ void synth_corrupt_kernel(uint8_t* __restrict__ base, uint64_t stride, uint32_t len, uint32_t n,
                                     uint64_t first, uint32_t corrupt_every) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n || len == 0) return;
    const uint64_t g = first + p;
    if (g % corrupt_every != corrupt_every - 1) return;
    base[(uint64_t)p * stride + (g * 7919u) % len] ^= 0xFF;
}

hipError_t launch_synth_fill(uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint64_t first,
                             uint64_t seed, uint32_t corrupt_every, hipStream_t stream) {
    if (n == 0 || len == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_fill_kernel, dim3(2048 * 4), dim3(256), 0, stream, base, stride, len, n, first, seed);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || corrupt_every == 0) return e;
    hipLaunchKernelGGL(synth_corrupt_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, base, stride, len, n, first,
                       corrupt_every);
    return hipGetLastError();
}

}  // namespace vx
