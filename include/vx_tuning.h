/*
 * vx_tuning.h — kernel-variant selection for A/B measurement (not part of
 * the drop-in boundary).  vx_sha1_device_uniform() always runs the default
 * (best measured) variant; this entry point lets tools/ and tests pin one.
 *   0 = default, 1 = lane-per-piece (one wave per 64 pieces does loads,
 *   schedule and rounds), 2 = producer/consumer split (a load+schedule wave
 *   feeds a rounds-only wave through an LDS ring), 3 / 4 = split with a 2- / 3-slot
 *   LDS ring (A/B of the ring protocol; 2 uses the default ring), 5 = split
 *   with one pair per CU (ragged only; what the planner picks for batches
 *   bound by their longest chain).
 */
#ifndef VX_TUNING_H
#define VX_TUNING_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

int vx_sha1_device_ragged_variant(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lens,
                                  const uint32_t* d_order, uint32_t n, void* d_digests, const void* d_expected,
                                  void* d_matched, void* stream, int variant);
/* Chunk rounds a context has launched on the resumable chunk paths (file
 * re-verify of pieces >= 2 chunks, strided host batches).
 * Tests use it to tell which path a batch took. */
struct vx_ctx;
uint64_t vx_tuning_chunk_rounds(const struct vx_ctx* ctx);
/* 64 KiB tiles the context's gather kernel has pulled from registered host
 * buffers (async / batch slots). */
uint64_t vx_tuning_gather_tiles(const struct vx_ctx* ctx);
/* Slots the context hashed with the zero-copy kernel (every piece registered
 * and aligned, read from host memory by the hash kernel itself, no gather;
 * DESIGN.md §6.5). */
uint64_t vx_tuning_zero_copy_slots(const struct vx_ctx* ctx);
/* ... of them, the slots hashed in the three-wave form (a loader wave beside
 * the pair; what the policy picks for slots of fewer than 128 pieces). */
uint64_t vx_tuning_zero_copy_loader_slots(const struct vx_ctx* ctx);
/* How a context with zero_copy = 1 hashes a slot of n registered, aligned
 * pieces of total_len bytes: 1 the zero-copy pair, 2 the zero-copy kernel
 * with a loader wave (n < 128, a latency-bound batch); 0 (gather + hash) is
 * only taken with zero_copy = 0.  Host-only. */
int vx_tuning_zero_copy_plan(uint32_t n, uint64_t total_len);
/* The zero-copy kernel on its own (A/B probes): piece i is d_lens[i] bytes at
 * the device-visible address d_srcs[i] (HBM, or a registered host buffer's
 * device mapping), 16-byte aligned; d_digests n x 20 B, d_expected /
 * d_matched optional.  loader = 0: the pair form, 1: the three-wave form.
 * Enqueue-only on `stream` (a hipStream_t or NULL). */
int vx_tuning_zero_copy_kernel(const uint64_t* d_srcs, const uint32_t* d_lens, uint32_t n, void* d_digests,
                               const void* d_expected, void* d_matched, int loader, void* stream);
/* Fault injection for tests: after k more successful piece submits (async or
 * inside a host batch), the next one fails with VX_ENOMEM without latching
 * the context, as a failed pinned-stage allocation does.  k < 0 turns it off. */
void vx_tuning_fail_submit_after(struct vx_ctx* ctx, int64_t k);
/* Fault injection for tests: after k more successful batch launches, the next
 * launch fails as a device error does (VX_EDEVICE, the context turns sticky):
 * the recovery path of INTEGRATION.md "Device failure".  k < 0 turns it off. */
void vx_tuning_fail_launch_after(struct vx_ctx* ctx, int64_t k);
/* The kernel vx_sha1_device_ragged_hint runs for a batch of n pieces whose
 * longest is max_len bytes, total_len bytes in all: 1 = lane, 2 = split,
 * 5 = split with one pair per CU (host-only). */
int vx_tuning_plan_ragged(uint32_t n, uint32_t max_len, uint64_t total_len);
/* The file re-verify's round boundaries for a window whose longest piece is
 * L bytes with chunk C (head/tail: ramp the first / last C bytes down to
 * C/4).  Writes up to max (offset, length) pairs to out
 * (2*max uint64_t) and returns the number of rounds (host-only). */
size_t vx_tuning_chunk_schedule(uint64_t L, uint64_t C, int head, int tail, uint64_t* out, size_t max);

/* Where the last vx_verify_files / vx_verify_files_range call on ctx spent
 * its time (bench.py records it per timed call).  Host times
 * are steady-clock; copy times are the GPU's own (events around each data
 * H2D) and exist only on the resumable chunk path (pieces >= 2 chunks). */
typedef struct vx_verify_trace {
    double wall_ms;        /* the whole call                                          */
    double read_busy_ms;   /* pread time summed over the reader threads               */
    double read_span_ms;   /* first read started -> last read finished                */
    double first_read_ms;  /* call start -> first read finished (nothing overlaps it) */
    double copy_busy_ms;   /* GPU-timed data copies, summed (chunk path)              */
    double copy_span_ms;   /* first copy start -> last copy end, GPU clock            */
    double tail_ms;        /* last round enqueued -> verdicts on the host             */
    uint64_t read_bytes;   /* bytes pread                                             */
    uint64_t copy_bytes;   /* bytes of the timed copies                               */
    uint32_t readers;      /* reader threads                                          */
    uint32_t rounds;       /* timed copies (chunk rounds)                             */
    uint64_t direct_bytes; /* of read_bytes, read with O_DIRECT (not cached; §6.1)    */
    uint64_t chunk_bytes;  /* chunk of the resumable rounds (0: whole-piece slots)    */
} vx_verify_trace;
int vx_tuning_last_verify(const struct vx_ctx* ctx, vx_verify_trace* out);

int vx_sha1_device_uniform_variant(const void* d_base, uint64_t stride, uint32_t len, uint32_t n, void* d_digests,
                                   const void* d_expected, void* d_matched, void* stream, int variant);

/* Shader-clock stamps (bench.py; vx_clock.hip): enqueue `blocks` one-wave
 * workgroups on `stream`; workgroup b writes d_out[3b..3b+2] = (shader cycle
 * counter, 100 MHz real-time counter, XCC id).  Two stamps bracketing a
 * stretch of work on one stream give each XCC's mean shader clock over it. */
int vx_tuning_clock_stamp(void* d_out, uint32_t blocks, void* stream);
/* The real-time counter's rate in kHz (hipDeviceAttributeWallClockRate). */
int vx_tuning_wall_clock_khz(int device);
/* Physical identity of HIP device `device`: its PCI bus id ("dddd:bb:dd.f",
 * NUL-terminated in bus_id[0..len), len >= 16) and 16-byte UUID. */
int vx_tuning_device_identity(int device, char* bus_id, size_t len, char* uuid16);

#ifdef __cplusplus
}
#endif
#endif
