/*
 * vx_synth.h — synthetic piece batches for tests and benchmarks (not part of
 * the drop-in boundary; the reference has no counterpart).
 *
 * Fills n pieces at d_base + i*stride (len bytes each) with the counter-based
 * splitmix64 stream of DESIGN.md "Synthetic pieces": piece i is global piece
 * first+i under `seed`; when corrupt_every != 0 every corrupt_every-th piece
 * gets one flipped byte.  The CPU oracle (oracle/sha1_oracle.c vxo_gen_piece)
 * regenerates the same bytes.  Enqueue-only on `stream`.
 */
#ifndef VX_SYNTH_H
#define VX_SYNTH_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

int vx_synth_fill(void* d_base, uint64_t stride, uint32_t len, uint32_t n, uint64_t first, uint64_t seed,
                  uint32_t corrupt_every, void* stream);

#ifdef __cplusplus
}
#endif
#endif
