// vx_kernels.h — internal launch interface between the C-ABI layer
// (vx_engine.hip) and the kernels (sha1_kernels.hip, vx_synth.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vx {

constexpr int kBlock = 256;  // 4 waves = one wave per SIMD of a CU
constexpr int kRing = 3;      // 128-byte groups in the ragged lane kernel's register ring
constexpr int kLaneRing = 4;  // ... and in the uniform lane kernel's (fenced, exact vmcnt)
constexpr int kPairBlock = 128;  // split kernel: consumer wave + producer wave

// Uniform-batch kernel variants (vx_tuning.h): 0 = default (best measured),
// 1 = lane-per-piece (one wave does everything), 2 = producer/consumer split.
// kSplitWide: the split kernel with one pair per CU (padded LDS), for
// batches bound by their longest chain with room to spare (plan_ragged).
enum UniformVariant {
    kUniformDefault = 0,
    kUniformLane = 1,
    kUniformSplit = 2,
    kSplitRing2 = 3,
    kSplitRing3 = 4,
    kSplitWide = 5
};
// LDS ring slots of the split kernels (sha1_kernels.hip "Ring protocol").
// 3: the producer runs two blocks ahead and the consumer prefetches the next
// block into registers while compressing (config 5 geometry 28.1 -> 26.6 ms,
// DESIGN.md §3.2).  2: the consumer reads each block at its top.  Variants
// 3 / 4 pin 2 / 3 slots for A/B runs.
constexpr int kSplitSlots = 3;
constexpr uint32_t kSplitMaxPieces = 16384;  // default picks split at or below this batch size

hipError_t launch_uniform(const uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint8_t* digests,
                          const uint8_t* expected, uint8_t* matched, hipStream_t stream, int variant = 0,
                          const uint32_t* exp_index = nullptr);
hipError_t launch_uniform_lane(const uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint8_t* digests,
                               const uint8_t* expected, uint8_t* matched, hipStream_t stream,
                               const uint32_t* exp_index = nullptr);
hipError_t launch_uniform_split(const uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint8_t* digests,
                                const uint8_t* expected, uint8_t* matched, hipStream_t stream,
                                const uint32_t* exp_index = nullptr);

// Lane (kUniformLane), split (kUniformSplit) or split with one pair per CU
// (kSplitWide) for a ragged batch, from its longest piece and total bytes
// (DESIGN.md §3.4).
int plan_ragged(uint32_t n, uint64_t max_len, uint64_t total_len);

hipError_t launch_ragged(const uint8_t* base, const uint64_t* offsets, const uint32_t* lens, const uint32_t* order,
                         uint32_t n, uint8_t* digests, const uint8_t* expected, uint8_t* matched,
                         hipStream_t stream, int variant = 0,
                          const uint32_t* exp_index = nullptr);
hipError_t launch_ragged_lane(const uint8_t* base, const uint64_t* offsets, const uint32_t* lens,
                              const uint32_t* order, uint32_t n, uint8_t* digests, const uint8_t* expected,
                              uint8_t* matched, hipStream_t stream, const uint32_t* exp_index = nullptr);
hipError_t launch_ragged_split(const uint8_t* base, const uint64_t* offsets, const uint32_t* lens,
                               const uint32_t* order, uint32_t n, uint8_t* digests, const uint8_t* expected,
                               uint8_t* matched, hipStream_t stream, const uint32_t* exp_index = nullptr);

// Resumable chunk kernel: lane j hashes bytes
// [poffs[j], poffs[j]+lens[j]) of piece pids[j] (total tlens[j]) from/to
// states[pid*5..]; the chunk that ends a piece emits digests/matched row pid
// (expected row pid).  Non-final chunk lengths must be multiples of 64.
hipError_t launch_chunk(const uint8_t* base, const uint64_t* offsets, const uint32_t* lens, uint32_t n,
                        const uint32_t* pids, const uint64_t* poffs, const uint64_t* tlens, uint32_t* states,
                        uint8_t* digests, const uint8_t* expected, uint8_t* matched, hipStream_t stream);

// Gather registered host pieces into a slot arena (vx_gather.hip, DESIGN.md
// §6.5): piece i (16-byte aligned device-mapped source src[i], length
// lens[i]) lands at arena + dst_off[i]; it owns 64 KiB tiles
// [tfirst[i], tfirst[i+1]) of the ntiles = tfirst[n] total.
uint32_t gather_tiles(uint32_t len);
hipError_t launch_gather(const uint64_t* src, const uint64_t* dst_off, const uint32_t* lens, const uint32_t* tfirst,
                         uint32_t n, uint32_t ntiles, uint8_t* arena, hipStream_t stream, uint32_t max_grid = 0);

// Zero-copy split kernel: piece i is read straight from
// registered host memory at its device-mapped address srcs[i] (16-byte
// aligned, lens[i] bytes; srcs[i] may be 0 when lens[i] == 0); digests /
// matched row i (expected row exp_index[i] when given).  loader: the
// three-wave form (a loader wave beside producer and consumer).
hipError_t launch_zero_copy(const uint64_t* srcs, const uint32_t* lens, uint32_t n, uint8_t* digests,
                            const uint8_t* expected, uint8_t* matched, bool loader, hipStream_t stream,
                            const uint32_t* exp_index = nullptr);

hipError_t launch_synth_fill(uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint64_t first,
                             uint64_t seed, uint32_t corrupt_every, hipStream_t stream);

}  // namespace vx
