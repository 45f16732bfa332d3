// sha1_kernels.hip — lane-per-piece SHA-1 kernels for MI355X (gfx950).
//
// Replaces the per-piece hash closure of vortex's pool
// (bittorrent/src/peer_comm/peer_connection.rs:1145-1158) and the bulk
// re-verify map (bittorrent/src/torrent.rs:724-740) for a whole batch of
// device-resident pieces at once.
//
// Mapping (DESIGN.md "Kernels"):
//  * lane j of the grid hashes one piece; a 256-thread workgroup = 4 waves =
//    one wave per SIMD of a CU.  65,536 pieces fill the chip exactly once
//    (256 CUs x 4 SIMDs x 64 lanes).
//  * each lane streams its piece in 128-byte groups (one L2 line, two SHA-1
//    blocks) with 8 x global_load_dwordx4, kept R-1 groups ahead of the
//    compression in a register ring so HBM latency hides behind ~1,200 VALU
//    per group; the loop bound is wave-uniform (scalar branch), the ring
//    indices are compile-time (no scratch).
//  * the tail (< 64 bytes + FIPS padding) is read byte-exactly, so no load
//    ever touches bytes past a piece's end.
//  * output: 20-byte big-endian digest per piece and, when an expected table
//    is given, a 0/1 verdict byte (DownloadedPiece::hash_matched).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sha1_device.hpp"
#include "vx_kernels.h"

namespace vx {

// A 128-byte line of zeros: the load target for lanes that have no full
// group to stream, so every issued load stays in bounds.
__device__ __attribute__((aligned(128))) uint4 g_zero_line[8];

__device__ __forceinline__ void load_group(uint4 (&dst)[8], const uint4* src) {
#pragma unroll
    for (int k = 0; k < 8; ++k) dst[k] = src[k];
}

__device__ __forceinline__ void compress_group(State& s, const uint4 (&g)[8]) {
    compress_le(s, g[0], g[1], g[2], g[3]);
    compress_le(s, g[4], g[5], g[6], g[7]);
}

// Stream `ng` 128-byte groups from src with an R-deep register ring.
// ng_wave: the wave-wide loop bound (== ng for uniform batches); lanes with
// ng < ng_wave keep issuing (clamped, in-bounds) loads and skip compression.
template <int R, bool kUniform>
__device__ __forceinline__ void stream_groups(State& s, const uint4* src, uint32_t ng, uint32_t ng_wave) {
    if (ng_wave == 0) return;
    const uint4* base = ng ? src : g_zero_line;
    const uint32_t last = ng ? ng - 1 : 0;
    uint4 ring[R][8];
#pragma unroll
    for (int r = 0; r < R - 1; ++r) {
        const uint32_t g = (uint32_t)r < last ? (uint32_t)r : last;
        load_group(ring[r], base + (size_t)g * 8);
    }
    for (uint32_t g0 = 0; g0 < ng_wave; g0 += R) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t gl_raw = g0 + r + R - 1;
            const uint32_t gl = gl_raw < last ? gl_raw : last;
            load_group(ring[(r + R - 1) % R], base + (size_t)gl * 8);
            if (kUniform) {
                if (g0 + r < ng_wave) compress_group(s, ring[r]);
            } else {
                if (g0 + r < ng) compress_group(s, ring[r]);
            }
        }
    }
}

template <bool kUniform>
__device__ __forceinline__ void hash_piece(State& s, const uint8_t* p, uint32_t len, uint32_t ng_wave) {
    const uint32_t nfull = len >> 6;
    const uint32_t ng = nfull >> 1;
    stream_groups<kRing, kUniform>(s, reinterpret_cast<const uint4*>(p), ng, ng_wave);
    const uint8_t* q = p + (size_t)ng * 128;
    if (nfull & 1) {
        const uint4* q4 = reinterpret_cast<const uint4*>(q);
        compress_le(s, q4[0], q4[1], q4[2], q4[3]);
        q += 64;
    }
    finalize(s, q, len & 63u, len);
}

__device__ __forceinline__ void emit(const State& s, uint32_t idx, uint8_t* __restrict__ digests,
                                     const uint8_t* __restrict__ expected, uint8_t* __restrict__ matched) {
    const uint32_t d0 = bswap(s.h0), d1 = bswap(s.h1), d2 = bswap(s.h2), d3 = bswap(s.h3), d4 = bswap(s.h4);
    if (digests) {
        uint32_t* o = reinterpret_cast<uint32_t*>(digests + (size_t)idx * 20);
        o[0] = d0;
        o[1] = d1;
        o[2] = d2;
        o[3] = d3;
        o[4] = d4;
    }
    if (expected && matched) {
        const uint32_t* x = reinterpret_cast<const uint32_t*>(expected + (size_t)idx * 20);
        const bool ok = (x[0] == d0) & (x[1] == d1) & (x[2] == d2) & (x[3] == d3) & (x[4] == d4);
        matched[idx] = ok ? 1 : 0;
    }
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t u = __shfl_xor(v, o, 64);
        v = u > v ? u : v;
    }
    return v;
}

__global__ __launch_bounds__(kBlock) void sha1_uniform_kernel(const uint8_t* __restrict__ base, uint64_t stride,
                                                              uint32_t len, uint32_t n,
                                                              uint8_t* __restrict__ digests,
                                                              const uint8_t* __restrict__ expected,
                                                              uint8_t* __restrict__ matched) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    // Lanes past n re-hash piece n-1 (in bounds, wave stays convergent) and
    // store nothing.
    const uint32_t pi = i < n ? i : n - 1;
    State s = iv();
    hash_piece<true>(s, base + (size_t)pi * stride, len, (len >> 7));
    if (i < n) emit(s, i, digests, expected, matched);
}

__global__ __launch_bounds__(kBlock) void sha1_ragged_kernel(const uint8_t* __restrict__ base,
                                                             const uint64_t* __restrict__ offsets,
                                                             const uint32_t* __restrict__ lens,
                                                             const uint32_t* __restrict__ order, uint32_t n,
                                                             uint8_t* __restrict__ digests,
                                                             const uint8_t* __restrict__ expected,
                                                             uint8_t* __restrict__ matched) {
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t jj = j < n ? j : n - 1;
    const uint32_t idx = order ? order[jj] : jj;
    const uint32_t len = lens[idx];
    const uint8_t* p = base + offsets[idx];
    const uint32_t ng_wave = __builtin_amdgcn_readfirstlane(wave_max(len >> 7));
    State s = iv();
    hash_piece<false>(s, p, len, ng_wave);
    if (j < n) emit(s, idx, digests, expected, matched);
}

hipError_t launch_uniform(const uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint8_t* digests,
                          const uint8_t* expected, uint8_t* matched, hipStream_t stream) {
    const uint32_t blocks = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(sha1_uniform_kernel, dim3(blocks), dim3(kBlock), 0, stream, base, stride, len, n, digests,
                       expected, matched);
    return hipGetLastError();
}

hipError_t launch_ragged(const uint8_t* base, const uint64_t* offsets, const uint32_t* lens, const uint32_t* order,
                         uint32_t n, uint8_t* digests, const uint8_t* expected, uint8_t* matched,
                         hipStream_t stream) {
    const uint32_t blocks = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(sha1_ragged_kernel, dim3(blocks), dim3(kBlock), 0, stream, base, offsets, lens, order, n,
                       digests, expected, matched);
    return hipGetLastError();
}

}  // namespace vx
