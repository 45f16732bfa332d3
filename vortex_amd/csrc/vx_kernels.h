// vx_kernels.h — internal launch interface between the C-ABI layer
// (vx_engine.hip) and the kernels (sha1_kernels.hip, vx_synth.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vx {

constexpr int kBlock = 256;  // 4 waves = one wave per SIMD of a CU
constexpr int kRing = 3;     // 128-byte groups in the per-lane register ring

hipError_t launch_uniform(const uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint8_t* digests,
                          const uint8_t* expected, uint8_t* matched, hipStream_t stream);

hipError_t launch_ragged(const uint8_t* base, const uint64_t* offsets, const uint32_t* lens, const uint32_t* order,
                         uint32_t n, uint8_t* digests, const uint8_t* expected, uint8_t* matched,
                         hipStream_t stream);

hipError_t launch_synth_fill(uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint64_t first,
                             uint64_t seed, uint32_t corrupt_every, hipStream_t stream);

}  // namespace vx
