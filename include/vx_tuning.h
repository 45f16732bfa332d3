/*
 * vx_tuning.h — measurement and test entry points, NOT part of the drop-in
 * boundary.  They are exported only by the test/tuning build
 * libvortex_amd_tuning.so (the same sources, linked with -DVX_TEST_HOOKS);
 * the library vortex links, libvortex_amd.so, exports vx_hash.h alone
 * (tests/test_abi.py checks both export lists with nm -D).  Unstable: these
 * may change in any release without an ABI version bump.
 *
 * Kernel variants (vx_sha1_device_*_variant): 0 = default (what
 * vx_sha1_device_uniform / _ragged run), 1 = lane-per-piece (one wave per 64
 * pieces does loads, schedule and rounds), 2 = producer/consumer split (a
 * load+schedule wave feeds a rounds-only wave through an LDS ring), 3 / 4 =
 * split with a 2- / 3-slot LDS ring (A/B of the ring protocol; 2 uses the
 * default ring), 5 = split with one pair per CU (ragged only; what the
 * planner picks for batches bound by their longest chain).
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
struct vx_ctx;
struct vx_split;
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
/* A/B of the file re-verify's copy placement: mode 1 (the
 * default) puts every chunk round's data H2D on the context's one
 * high-priority copy stream and its lane table on the slot's stream; 0 puts
 * both on the slot's stream behind a host wait for the previous round's copy
 * (round 4's form). */
void vx_tuning_verify_copy_stream(struct vx_ctx* ctx, int mode);
/* A/B of the pinned stages' memory: on = 1 allocates them as
 * 2 MiB-aligned transparent-huge-page mappings registered with hipHostRegister,
 * 0 with hipHostMalloc.  Idle stages are freed and reallocated on next use. */
void vx_tuning_stage_huge(struct vx_ctx* ctx, int on);
/* A/B of the split's rules for pieces of one chunk (vx_verify_files_split,
 * DESIGN.md §6.6): one_round = 1 (the default) lets their groups keep the
 * first group's rule until the rates are in, skips the tenth rule and reads
 * runs of them with one pread, 2 does the same piece by piece, 0 gives them
 * the multi-round pieces' rules; round_cap > 0 (default 64 MiB) caps
 * their rounds at that many bytes but no fewer than 1,024 lanes, 0 gives them
 * the slot's whole stage.  lag = 1 (the default) adds the learned lag to the
 * first group's T_engine, 0 keeps learning it without adding it.  learn = 1
 * (the default) starts each call from the median of the last five calls'
 * figures, 0 from their running mean (each call weighted 1/2). */
void vx_tuning_split_rules(struct vx_ctx* ctx, int one_round, uint64_t round_cap, int lag, int learn);
/* The kernel vx_sha1_device_ragged_hint runs for a batch of n pieces whose
 * longest is max_len bytes, total_len bytes in all: 1 = lane, 2 = split,
 * 5 = split with one pair per CU (host-only). */
int vx_tuning_plan_ragged(uint32_t n, uint32_t max_len, uint64_t total_len);
/* The file re-verify's round boundaries for a window whose longest piece is
 * L bytes with chunk C (head/tail: ramp the first / last C bytes down to
 * C/4).  Writes up to max (offset, length) pairs to out
 * (2*max uint64_t) and returns the number of rounds (host-only). */
size_t vx_tuning_chunk_schedule(uint64_t L, uint64_t C, int head, int tail, uint64_t* out, size_t max);
/* The engine's side of the split's claim word (vx_verify_files_split):
 * take up to k pieces from the top of the unclaimed range; returns the new
 * stop and (was, may be NULL) the stop before, so the pieces taken are
 * [returned, *was) (host-only). */
uint64_t vx_tuning_split_take_tail(struct vx_split* s, uint64_t k, uint64_t* was);
/* The last vx_verify_files_split call's decisions, one row of 13 doubles per
 * round it formed: ms since the call's start, the pool's rate (pieces/s), the
 * engine's intake rate (B/s), its chain per 64-byte block (ns), the predicted
 * remaining ms of the engine and of the pool with the group taken, unclaimed
 * pieces, the group taken, active lanes, the pool's finished pieces, the
 * decision mode (0 later round, 1 first, 2 forced), whether both sides'
 * rates were measured, and the learned lag (ms) inside the engine's time.
 * Writes up to max rows; returns the row count. */
size_t vx_tuning_last_split(const struct vx_ctx* ctx, double* out, size_t max);

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
