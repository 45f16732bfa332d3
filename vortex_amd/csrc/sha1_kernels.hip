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

#include <algorithm>
#include <cstdlib>
#include <stdint.h>

#include "sha1_consumer_asm.inc"
#include "sha1_device.hpp"
#include "vx_kernels.h"

namespace vx {

// A line of zeros: the load target for lanes that have no full group to
// stream, so every issued load stays in bounds (512 bytes: the zero-copy
// producer adds its 256-byte half offset after choosing it).
__device__ __attribute__((aligned(128))) uint4 g_zero_line[32];

__device__ __forceinline__ void load_group(uint4 (&dst)[8], const uint4* src) {
#pragma unroll
    for (int k = 0; k < 8; ++k) dst[k] = src[k];
}

// Issue a group's 8 loads strictly as [block A x4][block B x4] so counted
// vmcnt waits can release block A before block B lands (kFence variants).
__device__ __forceinline__ void load_group_ordered(uint4 (&dst)[8], const uint4* src) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = src[k];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 4; k < 8; ++k) dst[k] = src[k];
    __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void compress_group(State& s, const uint4 (&g)[8]) {
    compress_le(s, g[0], g[1], g[2], g[3]);
    compress_le(s, g[4], g[5], g[6], g[7]);
}

// Stream `ng` 128-byte groups from src with an R-deep register ring.
// ng_wave: the wave-wide loop bound (== ng for uniform batches); lanes with
// ng < ng_wave keep issuing (clamped, in-bounds) loads and skip compression.
template <int R, bool kUniform, bool kFence = false>
__device__ __forceinline__ void stream_groups(State& s, const uint4* src, uint32_t ng, uint32_t ng_wave) {
    if (ng_wave == 0) return;
    const uint4* base = ng ? src : g_zero_line;
    const uint32_t last = ng ? ng - 1 : 0;
    uint4 ring[R][8];
#pragma unroll
    for (int r = 0; r < R - 1; ++r) {
        const uint32_t g = (uint32_t)r < last ? (uint32_t)r : last;
        if (kFence && kUniform)
            load_group_ordered(ring[r], base + (size_t)g * 8);
        else
            load_group(ring[r], base + (size_t)g * 8);
    }
    if (kFence && kUniform) {
        // Branch-free steady state: whole R-group iterations with no guard
        // inside, so hipcc's waitcnt pass sees one straight block per trip and
        // emits exact counted vmcnt waits; loads fenced in issue order.
        uint32_t g0 = 0;
        for (; g0 + R <= ng_wave; g0 += R) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t gl_raw = g0 + r + R - 1;
                const uint32_t gl = gl_raw < last ? gl_raw : last;
                load_group_ordered(ring[(r + R - 1) % R], base + (size_t)gl * 8);
                compress_group(s, ring[r]);
            }
        }
        // remainder (< R groups), once per piece
#pragma unroll
        for (int r = 0; r < R - 1; ++r)
            if (g0 + r < ng_wave) compress_group(s, ring[r]);
        return;
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

template <bool kUniform, int R = kRing, bool kFence = false>
__device__ __forceinline__ void hash_piece(State& s, const uint8_t* p, uint32_t len, uint32_t ng_wave) {
    const uint32_t nfull = len >> 6;
    const uint32_t ng = nfull >> 1;
    stream_groups<R, kUniform, kFence>(s, reinterpret_cast<const uint4*>(p), ng, ng_wave);
    const uint8_t* q = p + (size_t)ng * 128;
    if (nfull & 1) {
        const uint4* q4 = reinterpret_cast<const uint4*>(q);
        compress_le(s, q4[0], q4[1], q4[2], q4[3]);
        q += 64;
    }
    finalize(s, q, len & 63u, len);
}

__device__ __forceinline__ void emit(const State& s, uint32_t idx, uint8_t* __restrict__ digests,
                                     const uint8_t* __restrict__ expected, uint8_t* __restrict__ matched,
                                     const uint32_t* __restrict__ exp_index = nullptr) {
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
        // exp_index: row of the device-resident piece table (vx_set_piece_table)
        const uint32_t row = exp_index ? exp_index[idx] : idx;
        const uint32_t* x = reinterpret_cast<const uint32_t*>(expected + (size_t)row * 20);
        const bool ok = (x[0] == d0) & (x[1] == d1) & (x[2] == d2) & (x[3] == d3) & (x[4] == d4);
        matched[idx] = ok ? 1 : 0;
    }
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t u = __shfl_xor(v, o, 64);
        v = u < v ? u : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t u = __shfl_xor(v, o, 64);
        v = u > v ? u : v;
    }
    return v;
}

template <int R, bool kAlias = false, bool kFence = false>
__global__ __launch_bounds__(kBlock) void sha1_uniform_kernel(const uint8_t* __restrict__ base, uint64_t stride,
                                                              uint32_t len, uint32_t n,
                                                              uint8_t* __restrict__ digests,
                                                              const uint8_t* __restrict__ expected,
                                                              uint8_t* __restrict__ matched,
                                                              const uint32_t* __restrict__ exp_index) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    // Lanes past n re-hash piece n-1 (in bounds, wave stays convergent) and
    // store nothing.
    const uint32_t pi = kAlias ? 0 : (i < n ? i : n - 1);  // kAlias: diagnostic, every lane reads piece 0
    State s = iv();
    hash_piece<true, R, kFence>(s, base + (size_t)pi * stride, len, (len >> 7));
    if (i < n) emit(s, i, digests, expected, matched, exp_index);
}

__global__ __launch_bounds__(kBlock) void sha1_ragged_kernel(const uint8_t* __restrict__ base,
                                                             const uint64_t* __restrict__ offsets,
                                                             const uint32_t* __restrict__ lens,
                                                             const uint32_t* __restrict__ order, uint32_t n,
                                                             uint8_t* __restrict__ digests,
                                                             const uint8_t* __restrict__ expected,
                                                             uint8_t* __restrict__ matched,
                                                             const uint32_t* __restrict__ exp_index) {
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t jj = j < n ? j : n - 1;
    const uint32_t idx = order ? order[jj] : jj;
    const uint32_t len = lens[idx];
    const uint8_t* p = base + offsets[idx];
    const uint32_t ng_wave = __builtin_amdgcn_readfirstlane(wave_max(len >> 7));
    State s = iv();
    hash_piece<false>(s, p, len, ng_wave);
    if (j < n) emit(s, idx, digests, expected, matched, exp_index);
}


// ---------------------------------------------------------------------------
// Producer/consumer ("split") uniform kernel.
//
// At 65,536 pieces the lane-per-piece kernel has exactly one wave per SIMD,
// and one wave can issue a VALU op only every ~4 cycles while a SIMD-32 can
// retire a wave64 op every 2 (MI355X_MICROARCH.md, 'vector-instruction ISSUE
// cost').  So each 64-piece group gets TWO waves on the chip: a consumer wave
// runs only the 80 rounds (5 VALU/round: alignbit, bitop3, 2x add3,
// alignbit), a producer wave does everything else — HBM loads, byte swaps and
// the W[16..79] schedule (3 VALU/word) — and hands each block's 80 words to
// the consumer through a 2-slot LDS ring ([slot][t/4][lane] uint4: one
// ds_write_b128 / ds_read_b128 per 4 words, lane-contiguous, conflict-free).
// One 128-thread workgroup = one pair; 40 KiB LDS → 4 pairs per CU.
// Barrier protocol (both waves pass nb+1 barriers):
//   producer: for b { P(b) -> slot b&1; sync }  sync
//   consumer: sync  for b { C(b) <- slot b&1; sync }
// so P(b+1) overlaps C(b) on the other slot.
// ---------------------------------------------------------------------------

__device__ __forceinline__ void expand_store(uint32_t (&w)[16], uint4 (*dst)[64], int lane) {
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[q][lane] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
#pragma unroll
    for (int q = 4; q < 20; ++q) {
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = 4 * q + j;
            const uint32_t x = rotl(VX_XOR2(VX_PAR(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]), w[t & 15]), 1);
            w[t & 15] = x;
            v[j] = x;
        }
        dst[q][lane] = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

__device__ __forceinline__ void rounds_lds(State& s, const uint4 (*src)[64], int lane) {
    uint32_t a = s.h0, b = s.h1, c = s.h2, d = s.h3, e = s.h4;
#pragma unroll
    for (int q = 0; q < 20; ++q) {
        const uint4 w4 = src[q][lane];
        const uint32_t wq[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = 4 * q + j;
            uint32_t f, k;
            if (t < 20) {
                f = VX_CH(b, c, d);
                k = kK0;
            } else if (t < 40) {
                f = VX_PAR(b, c, d);
                k = kK1;
            } else if (t < 60) {
                f = VX_MAJ(b, c, d);
                k = kK2;
            } else {
                f = VX_PAR(b, c, d);
                k = kK3;
            }
            const uint32_t tmp = rotl(a, 5) + f + e + k + wq[j];
            e = d;
            d = c;
            c = rotl(b, 30);
            b = a;
            a = tmp;
        }
    }
    s.h0 += a;
    s.h1 += b;
    s.h2 += c;
    s.h3 += d;
    s.h4 += e;
}

// ---------------------------------------------------------------------------
// Ring protocol between the producer and consumer waves, S slots of 80 words.
//  S = 2: the producer is one block ahead; the consumer reads block b from
//         LDS at the top of block b and stalls on those 20 ds_read_b128.
//  S = 3: the producer is two blocks ahead, so the consumer reads block b+1
//         into a second register set WHILE it compresses block b: no LDS
//         wait on the chain (60 KiB per pair: 2 pairs per CU instead of 4).
// Both waves pass 1 + nb_wave barriers:
//   producer: for b { P(b) -> slot(b); publish(b) }  producer_done
//   consumer: consume (initial barrier, then one per block)
// ---------------------------------------------------------------------------
template <int S>
struct RingLds {
    uint4 w[S][20][64];
};

template <int S>
__device__ __forceinline__ uint32_t ring_slot(uint32_t b) {
    return S == 2 ? (b & 1u) : (b % 3u);
}

// Producer: block b is in its slot.  S = 3 publishes blocks 0 and 1 together.
template <int S>
__device__ __forceinline__ void publish(uint32_t b) {
    if (S == 2 || b >= 1) __syncthreads();
}

template <int S>
__device__ __forceinline__ void producer_done(uint32_t nb_wave) {
    if (S == 2) {
        __syncthreads();
    } else if (nb_wave) {
        __syncthreads();
        __syncthreads();
    }
}

__device__ __forceinline__ void load_w(uint4 (&r)[20], const uint4 (*src)[64], int lane) {
#pragma unroll
    for (int q = 0; q < 20; ++q) r[q] = src[q][lane];
}

__device__ __forceinline__ void rounds_regs(State& s, const uint4 (&w)[20]) {
    uint32_t a = s.h0, b = s.h1, c = s.h2, d = s.h3, e = s.h4;
#pragma unroll
    for (int q = 0; q < 20; ++q) {
        const uint32_t wq[4] = {w[q].x, w[q].y, w[q].z, w[q].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = 4 * q + j;
            uint32_t f, k;
            if (t < 20) {
                f = VX_CH(b, c, d);
                k = kK0;
            } else if (t < 40) {
                f = VX_PAR(b, c, d);
                k = kK1;
            } else if (t < 60) {
                f = VX_MAJ(b, c, d);
                k = kK2;
            } else {
                f = VX_PAR(b, c, d);
                k = kK3;
            }
            const uint32_t tmp = rotl(a, 5) + f + e + k + wq[j];
            e = d;
            d = c;
            c = rotl(b, 30);
            b = a;
            a = tmp;
        }
    }
    s.h0 += a;
    s.h1 += b;
    s.h2 += c;
    s.h3 += d;
    s.h4 += e;
}

// Consumer for the 3-slot ring as ONE asm body (sha1_consumer_asm.inc,
// generated and checked by tools/gen_sha1_rounds.py): hipcc's own schedule
// and registers for the rounds ran a lone wave at ~4.5 cycles per VALU,
// the fixed stream at ~4.06 including the ring reads
// (a round-2 scheduling probe, EXPERIMENTS.md §3.2).  The asm holds the
// block loop, the ring reads (block b+1's 20 ds_read_b128 in a burst at the
// top of block b into the other of two word sets), the barriers (1 + nb_wave,
// as the C++ consumer) and, with kSelect, the ragged phase-2 commit for
// lanes with b < nb.  In the kernels it is 3-7 % faster per block than
// hipcc's consumer (profiles/r02/consumer_asm/).  Build with
// -DVX_CONSUMER_CC for the compiler-scheduled consumer (A/B).
template <bool kSelect>
__device__ __forceinline__ void consume_asm(State& s, const uint4* lds_lane, uint32_t nb_wave, uint32_t b1,
                                            uint32_t nb) {
    // LDS byte address: the low 32 bits of the generic address of a
    // __shared__ object are its offset in the workgroup's LDS.
    const uint32_t addr = (uint32_t)(uintptr_t)lds_lane;
    if (kSelect)
        asm volatile(VX_CONSUMER_SELECT_ASM
                     : "+v"(s.h0), "+v"(s.h1), "+v"(s.h2), "+v"(s.h3), "+v"(s.h4)
                     : "v"(addr), "s"(nb_wave), "s"(b1), "v"(nb)
                     : VX_CONSUMER_SELECT_ASM_CLOBBERS, "memory");
    else
        asm volatile(VX_CONSUMER_ASM
                     : "+v"(s.h0), "+v"(s.h1), "+v"(s.h2), "+v"(s.h3), "+v"(s.h4)
                     : "v"(addr), "s"(nb_wave), "s"(b1), "v"(nb)
                     : VX_CONSUMER_ASM_CLOBBERS, "memory");
}

// Consumer: compress blocks [0, nb_wave).  kSelect: blocks >= b1 commit only
// for lanes with b < nb (ragged phase 2); otherwise b1 == nb_wave == nb.
template <int S, bool kSelect>
__device__ __forceinline__ void consume(State& s, RingLds<S>& lds, int lane, uint32_t nb_wave, uint32_t b1,
                                        uint32_t nb) {
    if (S == 2) {
        __syncthreads();
        for (uint32_t b = 0; b < b1; ++b) {
            rounds_lds(s, lds.w[b & 1], lane);
            __syncthreads();
        }
        if (kSelect) {
            for (uint32_t b = b1; b < nb_wave; ++b) {
                State t = s;
                rounds_lds(t, lds.w[b & 1], lane);
                if (b < nb) s = t;
                __syncthreads();
            }
        }
        return;
    }
#ifndef VX_CONSUMER_CC
    if (S == 3) {
        consume_asm<kSelect>(s, &lds.w[0][0][lane], nb_wave, b1, nb);
        return;
    }
#endif
    if (nb_wave == 0) return;
    auto step = [&](uint32_t b, const uint4 (&r)[20]) {
        if (!kSelect || b < b1) {
            rounds_regs(s, r);
        } else {
            State t = s;
            rounds_regs(t, r);
            if (b < nb) s = t;
        }
        // The state must exist before the next barrier: without this hipcc
        // sinks the whole block's rounds below the s_barrier (they only feed
        // later blocks), and the barrier's lgkmcnt(0) then waits on the
        // freshly issued reads with nothing to overlap them.
        asm volatile("" : "+v"(s.h0), "+v"(s.h1), "+v"(s.h2), "+v"(s.h3), "+v"(s.h4));
    };
    // sched_barrier(0) keeps the scheduler from moving the next block's
    // ds_reads into or past the rounds.
    uint4 r0[20], r1[20];
    __syncthreads();
    load_w(r0, lds.w[0], lane);
    // Drain block 0's reads before the loop: hipcc's waitcnt pass merges the
    // loop entry with the back edge, and with these 20 reads still pending on
    // entry it put an lgkmcnt(14) on the next block's fresh reads in EVERY
    // trip (the 4-bit counter saturates).  lgkmcnt(0), other counters max.
    __builtin_amdgcn_s_waitcnt(0xC07F);
    uint32_t b = 0;
    for (; b + 2 <= nb_wave; b += 2) {
        load_w(r1, lds.w[ring_slot<S>(b + 1)], lane);
        __builtin_amdgcn_sched_barrier(0);
        step(b, r0);
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
        if (b + 2 < nb_wave) load_w(r0, lds.w[ring_slot<S>(b + 2)], lane);
        __builtin_amdgcn_sched_barrier(0);
        step(b + 1, r1);
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
    }
    if (b < nb_wave) {
        step(b, r0);
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
    }
}

__device__ __forceinline__ void le_words(uint32_t (&w)[16], const uint4& q0, const uint4& q1, const uint4& q2,
                                         const uint4& q3) {
    const uint4 q[4] = {q0, q1, q2, q3};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        w[4 * k + 0] = bswap(q[k].x);
        w[4 * k + 1] = bswap(q[k].y);
        w[4 * k + 2] = bswap(q[k].z);
        w[4 * k + 3] = bswap(q[k].w);
    }
}

// Tail words of FIPS 180-4 padding (same byte rules as finalize()).
__device__ __forceinline__ void tail_words(uint32_t (&w)[16], const uint8_t* q, uint32_t rem) {
    const uint32_t* q32 = reinterpret_cast<const uint32_t*>(q);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t off = 4u * k;
        uint32_t v = 0;
        if (off + 4 <= rem) {
            v = q32[k];
        } else if (off < rem) {
            for (uint32_t j = 0; off + j < rem; ++j) v |= (uint32_t)q[off + j] << (8 * j);
        }
        if (rem >= off && rem < off + 4) v |= 0x80u << (8 * (rem - off));
        w[k] = bswap(v);
    }
}

template <int S>
__global__ __launch_bounds__(kPairBlock) void sha1_split_kernel(const uint8_t* __restrict__ base, uint64_t stride,
                                                                uint32_t len, uint32_t n,
                                                                uint8_t* __restrict__ digests,
                                                                const uint8_t* __restrict__ expected,
                                                                uint8_t* __restrict__ matched,
                                                                const uint32_t* __restrict__ exp_index) {
    __shared__ RingLds<S> lds;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t i = blockIdx.x * 64 + lane;
    const uint32_t pi = i < n ? i : n - 1;
    const uint8_t* p = base + (size_t)pi * stride;
    const uint32_t nfull = len >> 6;
    const uint32_t rem = len & 63u;
    const uint32_t nb = nfull + (rem <= 55 ? 1u : 2u);

    if (wave == 1) {
        // ---------------- producer ----------------
        uint32_t b = 0;
        uint32_t w[16];
        const uint32_t ng = len >> 7;
        const uint4* src = reinterpret_cast<const uint4*>(p);
        if (ng) {
            constexpr int R = kRing;
            const uint32_t last = ng - 1;
            uint4 ring[R][8];
#pragma unroll
            for (int r = 0; r < R - 1; ++r) {
                const uint32_t g = (uint32_t)r < last ? (uint32_t)r : last;
                load_group(ring[r], src + (size_t)g * 8);
            }
            for (uint32_t g0 = 0; g0 < ng; g0 += R) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t gl_raw = g0 + r + R - 1;
                    const uint32_t gl = gl_raw < last ? gl_raw : last;
                    load_group(ring[(r + R - 1) % R], src + (size_t)gl * 8);
                    if (g0 + r < ng) {
                        le_words(w, ring[r][0], ring[r][1], ring[r][2], ring[r][3]);
                        expand_store(w, lds.w[ring_slot<S>(b)], lane);
                        publish<S>(b);
                        ++b;
                        le_words(w, ring[r][4], ring[r][5], ring[r][6], ring[r][7]);
                        expand_store(w, lds.w[ring_slot<S>(b)], lane);
                        publish<S>(b);
                        ++b;
                    }
                }
            }
        }
        const uint8_t* q = p + (size_t)ng * 128;
        if (nfull & 1) {
            const uint4* q4 = reinterpret_cast<const uint4*>(q);
            le_words(w, q4[0], q4[1], q4[2], q4[3]);
            expand_store(w, lds.w[ring_slot<S>(b)], lane);
            publish<S>(b);
            ++b;
            q += 64;
        }
        tail_words(w, q, rem);
        const uint32_t bits_hi = (uint32_t)(((uint64_t)len * 8u) >> 32);
        const uint32_t bits_lo = (uint32_t)((uint64_t)len * 8u);
        if (rem <= 55) {
            w[14] = bits_hi;
            w[15] = bits_lo;
            expand_store(w, lds.w[ring_slot<S>(b)], lane);
            publish<S>(b);
        } else {
            expand_store(w, lds.w[ring_slot<S>(b)], lane);
            publish<S>(b);
            ++b;
#pragma unroll
            for (int k = 0; k < 14; ++k) w[k] = 0;
            w[14] = bits_hi;
            w[15] = bits_lo;
            expand_store(w, lds.w[ring_slot<S>(b)], lane);
            publish<S>(b);
        }
        producer_done<S>(nb);
    } else {
        // ---------------- consumer ----------------
        State s = iv();
        consume<S, false>(s, lds, lane, nb, nb, nb);
        if (i < n) emit(s, i, digests, expected, matched, exp_index);
    }
}

template <int S>
hipError_t launch_uniform_split_s(const uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint8_t* digests,
                                  const uint8_t* expected, uint8_t* matched, hipStream_t stream,
                                  const uint32_t* exp_index) {
    const uint32_t blocks = (n + 63) / 64;
    hipLaunchKernelGGL(sha1_split_kernel<S>, dim3(blocks), dim3(kPairBlock), 0, stream, base, stride, len, n,
                       digests, expected, matched, exp_index);
    return hipGetLastError();
}

hipError_t launch_uniform_split(const uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint8_t* digests,
                                const uint8_t* expected, uint8_t* matched, hipStream_t stream,
                                const uint32_t* exp_index) {
    return launch_uniform_split_s<kSplitSlots>(base, stride, len, n, digests, expected, matched, stream, exp_index);
}


// ---------------------------------------------------------------------------
// Ragged producer/consumer kernel: per-lane offsets/lengths, same two-wave
// split as sha1_split_kernel.  The wave-uniform trip count is the wave's
// longest piece (in blocks incl. padding); the producer feeds every lane
// data blocks, then its 1-2 padding blocks, then zeros, and the consumer
// commits a block's result only for lanes still inside their piece (a
// v_cndmask select, no divergent rounds).  Pieces should arrive sorted by
// descending length (vx_sort_order) so each wave's lanes finish together.
// ---------------------------------------------------------------------------
constexpr int kBlockRing = 6;  // 64-byte blocks of loads in flight per lane

__device__ __forceinline__ void load_block(uint4 (&dst)[4], const uint4* src) {
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = src[k];
}

// Words of padding block k (0 or 1) of a piece whose tail has `rem` bytes at q.
__device__ __forceinline__ void pad_words(uint32_t (&w)[16], const uint8_t* q, uint32_t rem, uint64_t len,
                                          uint32_t k) {
    const uint32_t bits_hi = (uint32_t)((len * 8u) >> 32);
    const uint32_t bits_lo = (uint32_t)(len * 8u);
    if (k == 0) {
        tail_words(w, q, rem);
        if (rem <= 55) {
            w[14] = bits_hi;
            w[15] = bits_lo;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = 0;
        if (k == 1 && rem > 55) {
            w[14] = bits_hi;
            w[15] = bits_lo;
        }
    }
}

// kChunked: resumable hashing of one chunk per lane.  SHA-1's
// chaining state is 20 bytes, so a piece can be compressed chunk by chunk
// across launches: lane j hashes bytes [poffs[j], poffs[j]+lens[j]) of piece
// pids[j] (total length tlens[j]) starting from states[pid] (or the IV when
// poffs[j] == 0); a chunk that ends the piece pads with the piece's total
// length and emits digest/verdict for row pid, any other chunk (a multiple of
// 64 bytes) stores the state back.
template <bool kChunked, int S>
__global__ __launch_bounds__(kPairBlock) void sha1_ragged_split_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets, const uint32_t* __restrict__ lens,
    const uint32_t* __restrict__ order, uint32_t n, uint8_t* __restrict__ digests,
    const uint8_t* __restrict__ expected, uint8_t* __restrict__ matched, const uint32_t* __restrict__ exp_index,
    const uint32_t* __restrict__ pids, const uint64_t* __restrict__ poffs, const uint64_t* __restrict__ tlens,
    uint32_t* __restrict__ states) {
    __shared__ RingLds<S> lds;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t j = blockIdx.x * 64 + lane;
    const uint32_t jj = j < n ? j : n - 1;
    const uint32_t idx = order ? order[jj] : jj;
    const uint32_t len = lens[idx];
    const uint8_t* p = base + offsets[idx];
    const uint32_t pid = kChunked ? pids[idx] : idx;
    const uint64_t poff = kChunked ? poffs[idx] : 0;
    const uint64_t tlen = kChunked ? tlens[idx] : len;
    const bool final_chunk = poff + len == tlen;
    const uint32_t nfull = len >> 6;
    const uint32_t rem = len & 63u;
    const uint32_t nb = final_chunk ? nfull + (rem <= 55 ? 1u : 2u) : nfull;
    const uint32_t nb_wave = __builtin_amdgcn_readfirstlane(wave_max(nb));
    // Phase 1 [0, b1): every lane of the wave has a full data block, so the
    // producer streams a fenced block ring with no per-lane branch and the
    // consumer commits unconditionally.  Phase 2 [b1, nb_wave): per-lane
    // data / padding / idle (a few blocks when the wave's lengths differ).
    constexpr int R = kBlockRing;
    const uint32_t nfull_min = __builtin_amdgcn_readfirstlane(wave_min(nfull));
    const uint32_t b1 = nfull_min / R * R;

    if (wave == 1) {
        // ---------------- producer ----------------
        const uint4* src = nfull ? reinterpret_cast<const uint4*>(p) : g_zero_line;
        const uint32_t last = nfull ? nfull - 1 : 0;
        const uint8_t* q = p + (size_t)nfull * 64;
        uint32_t w[16];
        if (b1) {
            uint4 ring[R][4];
#pragma unroll
            for (int r = 0; r < R - 1; ++r) {
                __builtin_amdgcn_sched_barrier(0);
                load_block(ring[r], src + (size_t)r * 4);
            }
            for (uint32_t b0 = 0; b0 < b1; b0 += R) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t bl_raw = b0 + r + R - 1;
                    const uint32_t bl = bl_raw < last ? bl_raw : last;
                    __builtin_amdgcn_sched_barrier(0);
                    load_block(ring[(r + R - 1) % R], src + (size_t)bl * 4);
                    __builtin_amdgcn_sched_barrier(0);
                    le_words(w, ring[r][0], ring[r][1], ring[r][2], ring[r][3]);
                    expand_store(w, lds.w[ring_slot<S>(b0 + r)], lane);
                    publish<S>(b0 + r);
                }
            }
        }
        if (b1 < nb_wave) {
            // Phase 2: same fenced ring (clamped to each lane's last data
            // block), then a per-lane select between the data words, the
            // padding words (built once, before the loop: no byte loads in
            // the loop) and zeros for lanes already past their piece.
            uint32_t padw[16];
            tail_words(padw, q, rem);
            const uint32_t bits_hi = (uint32_t)((tlen * 8u) >> 32);
            const uint32_t bits_lo = (uint32_t)(tlen * 8u);
            if (rem <= 55) {
                padw[14] = bits_hi;
                padw[15] = bits_lo;
            }
            uint4 ring[R][4];
#pragma unroll
            for (int r = 0; r < R - 1; ++r) {
                const uint32_t bl_raw = b1 + r;
                const uint32_t bl = bl_raw < last ? bl_raw : last;
                __builtin_amdgcn_sched_barrier(0);
                load_block(ring[r], src + (size_t)bl * 4);
            }
            for (uint32_t b0 = b1; b0 < nb_wave; b0 += R) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t b = b0 + r;
                    const uint32_t bl_raw = b + R - 1;
                    const uint32_t bl = bl_raw < last ? bl_raw : last;
                    __builtin_amdgcn_sched_barrier(0);
                    load_block(ring[(r + R - 1) % R], src + (size_t)bl * 4);
                    __builtin_amdgcn_sched_barrier(0);
                    if (b < nb_wave) {  // wave-uniform
                        le_words(w, ring[r][0], ring[r][1], ring[r][2], ring[r][3]);
                        const bool is_pad0 = b == nfull;
                        const bool is_pad1 = b == nfull + 1;
#pragma unroll
                        for (int k = 0; k < 16; ++k) {
                            uint32_t v = b < nfull ? w[k] : 0u;
                            v = is_pad0 ? padw[k] : v;
                            if (k >= 14) v = (is_pad1 && rem > 55) ? (k == 14 ? bits_hi : bits_lo) : v;
                            w[k] = v;
                        }
                        expand_store(w, lds.w[ring_slot<S>(b)], lane);
                        publish<S>(b);
                    }
                }
            }
        }
        producer_done<S>(nb_wave);
    } else {
        // ---------------- consumer ----------------
        State s = iv();
        if (kChunked && poff != 0) {
            const uint32_t* st = states + (size_t)pid * 5;
            s = State{st[0], st[1], st[2], st[3], st[4]};
        }
        consume<S, true>(s, lds, lane, nb_wave, b1, nb);
        if (j < n) {
            if (!kChunked || final_chunk) {
                emit(s, pid, digests, expected, matched, exp_index);
            } else {
                uint32_t* st = states + (size_t)pid * 5;
                st[0] = s.h0;
                st[1] = s.h1;
                st[2] = s.h2;
                st[3] = s.h3;
                st[4] = s.h4;
            }
        }
    }
}

// wide: unused dynamic LDS on top of the ring (60 KiB + 40 KiB > half of a
// CU's 160 KiB), so each CU holds one pair.  On a chain-bound batch the pairs
// hashing the longest pieces then keep their CU to themselves: config 3 56.8
// -> 53.4 ms (282 -> 300 GiB/s), the rest of its 16 GiB still done in time
// at half the split kernel's throughput.
constexpr uint32_t kWidePadLds = 40 * 1024;

template <int S>
hipError_t launch_ragged_split_s(const uint8_t* base, const uint64_t* offsets, const uint32_t* lens,
                                 const uint32_t* order, uint32_t n, uint8_t* digests, const uint8_t* expected,
                                 uint8_t* matched, hipStream_t stream, const uint32_t* exp_index,
                                 bool wide = false) {
    const uint32_t blocks = (n + 63) / 64;
    hipLaunchKernelGGL((sha1_ragged_split_kernel<false, S>), dim3(blocks), dim3(kPairBlock),
                       wide ? kWidePadLds : 0u, stream, base,
                       offsets, lens, order, n, digests, expected, matched, exp_index, nullptr, nullptr, nullptr,
                       nullptr);
    return hipGetLastError();
}

hipError_t launch_ragged_split(const uint8_t* base, const uint64_t* offsets, const uint32_t* lens,
                               const uint32_t* order, uint32_t n, uint8_t* digests, const uint8_t* expected,
                               uint8_t* matched, hipStream_t stream, const uint32_t* exp_index) {
    return launch_ragged_split_s<kSplitSlots>(base, offsets, lens, order, n, digests, expected, matched, stream,
                                              exp_index);
}

hipError_t launch_chunk(const uint8_t* base, const uint64_t* offsets, const uint32_t* lens, uint32_t n,
                        const uint32_t* pids, const uint64_t* poffs, const uint64_t* tlens, uint32_t* states,
                        uint8_t* digests, const uint8_t* expected, uint8_t* matched, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t blocks = (n + 63) / 64;
    hipLaunchKernelGGL((sha1_ragged_split_kernel<true, kSplitSlots>), dim3(blocks), dim3(kPairBlock), 0, stream, base, offsets,
                       lens, nullptr, n, digests, expected, matched, nullptr, pids, poffs, tlens, states);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Zero-copy split kernel: the async path's slots of
// registered pieces are hashed straight out of host memory through the
// pieces' device mappings (srcs[i], 16-byte aligned), with no gather kernel,
// so a slot's PCIe transfer overlaps its own hashing instead of preceding it.
// Same pair and ring protocol as sha1_ragged_split_kernel; the producer's
// loads differ.  Over PCIe the load SHAPE decides the rate
// (tools/native/zc_pattern_probe.hip): one lane per piece, as the HBM kernels
// load, reaches 28-31 GiB/s; 16 lanes per piece, 256 contiguous bytes of each
// of 4 pieces per wave instruction, 51-53 GiB/s once ~1 MiB is in flight.
//
// A pair hashes kZcPieces = 32 pieces (lanes 32-63 mirror lanes 0-31 and
// emit nothing): the chain per block is the same at 32 or 64 live lanes, the
// async slots leave most CUs idle, and so every piece gets twice the bytes in
// flight — a tile is 8 blocks (512 B) of all 32 pieces, 16 wave instructions,
// and two tiles (32 KiB) are in flight per producer wave, 1 KiB per piece.
// A landed tile is transposed through a 16.5 KiB LDS stage (chunk c of piece
// p at [c][p], rows padded to 33 slots: conflict-free both ways, and every
// access is one base register plus an immediate offset) to the lane that
// owns the piece.  Chunks past a piece's full blocks load the device zero line, so no
// load reaches past a piece; the < 64-byte tail and the padding come from the
// lane's own bytes (tail_words), as in the ragged kernel's phase 2.
// ---------------------------------------------------------------------------
constexpr uint32_t kZcPieces = 32;      // pieces per pair
constexpr uint32_t kZcTileBlocks = 8;   // 64-byte blocks per piece per tile
constexpr uint32_t kZcChunks = kZcTileBlocks * 4;  // 16-byte chunks per piece per tile

typedef uint32_t U32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) U32x4 GlobalU32x4;

// Load instruction k of tile t: 16 bytes at zb[k & 7] + t*512 (+256 for
// the second half, k >= 8) when that chunk lies inside the piece's full
// blocks (t*512 (+256) < zl[k & 7]), else the zero line.  zb and zl stay in
// VGPRs: read from LDS they put two dependent LDS round trips in front of
// every block's loads.  Explicitly global loads: the pointers come from
// memory, and as flat loads they would also count in lgkmcnt, which every
// ring barrier drains.
__device__ __forceinline__ uint4 zc_load(int k, const uint64_t (&zb)[8], const uint32_t (&zl)[8], uint32_t t) {
    const uint32_t o = t * (kZcTileBlocks * 64) + (k >= 8 ? 256u : 0u);
    const uint64_t zero = reinterpret_cast<uint64_t>(g_zero_line);
    const uint64_t a = (o < zl[k & 7] ? zb[k & 7] + t * (kZcTileBlocks * 64) : zero) + (k >= 8 ? 256u : 0u);
    const U32x4 v = *reinterpret_cast<GlobalU32x4*>(a);  // a native vector load: a uint4 struct copy from AS1
    return make_uint4(v.x, v.y, v.z, v.w);                 // became a memcpy that kept the tiles in scratch
}

// All 16 loads of tile t (the prologue).
__device__ __forceinline__ void zc_load_tile(uint4 (&r)[16], const uint64_t (&zb)[8], const uint32_t (&zl)[8],
                                             uint32_t t) {
#pragma unroll
    for (int k = 0; k < 16; ++k) r[k] = zc_load(k, zb, zl, t);
}

// Two of tile t's 16 loads (instructions k0 and k0 + 1): the producer
// spreads a tile's loads and stage writes over the 8 blocks of the tile
// before it, so no block carries them all.
__device__ __forceinline__ void zc_load_pair(uint4 (&r)[16], int k0, const uint64_t (&zb)[8],
                                             const uint32_t (&zl)[8], uint32_t t) {
    r[k0] = zc_load(k0, zb, zl, t);
    r[k0 + 1] = zc_load(k0 + 1, zb, zl, t);
}

// The loading side's setup: this lane's sources and limits, tiles 0-2 in
// flight, tile 0 staged.  Load instruction k covers pieces 4(k & 7) .. +3 (16
// lanes each) and the (k >> 3)-th 256-byte half of the tile: this lane moves
// chunk c16 + 16(k >> 3) of piece 4(k & 7) + (lane >> 4), so it keeps one
// source and one limit per piece group g = k & 7: the chunk at tile offset o
// is data iff o + 16 c16 + 16 <= the piece's full-block bytes, i.e. o < zl[g].
__device__ __forceinline__ void zc_setup(uint64_t (&zb)[8], uint32_t (&zl)[8], uint4 (&ra)[16], uint4 (&rb)[16],
                                         uint4 (&stage)[2][kZcChunks][kZcPieces + 1], const uint64_t* srcs,
                                         const uint32_t* lens, uint32_t n, uint32_t g0, int lane) {
    const uint32_t c16 = lane & 15;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        const uint32_t pk = g0 + 4 * g + (lane >> 4);
        const uint32_t pkk = pk < n ? pk : n - 1;
        const uint32_t full = pk < n ? (lens[pkk] >> 6) * 64u : 0u;
        zb[g] = srcs[pkk] + 16 * c16;
        zl[g] = full >= 16 * c16 + 16 ? full - 16 * c16 - 15 : 0u;
    }
    zc_load_tile(ra, zb, zl, 0);
    zc_load_tile(rb, zb, zl, 1);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t p = 4 * (k & 7) + (lane >> 4), c = c16 + 16 * (k >> 3);
        stage[0][c][p] = ra[k];
    }
    zc_load_tile(ra, zb, zl, 2);
}

// kLoader = false: a pair (consumer wave 0, producer wave 1 that loads,
// transposes and expands).  kLoader = true: a third wave (2) takes the loads
// and stage writes, so the expanding producer carries only what the split
// kernel's producer does; all three pass the same barriers (one extra at the
// start, once tile 0 is staged).
template <int S, bool kLoader>
__global__ __launch_bounds__(kLoader ? 3 * 64 : kPairBlock) void sha1_zc_split_kernel(
    const uint64_t* __restrict__ srcs, const uint32_t* __restrict__ lens, uint32_t n, uint8_t* __restrict__ digests,
    const uint8_t* __restrict__ expected, uint8_t* __restrict__ matched, const uint32_t* __restrict__ exp_index) {
    __shared__ RingLds<S> lds;
    __shared__ uint4 stage[2][kZcChunks][kZcPieces + 1];  // tile t in stage[t & 1]; rows padded to 33 slots
    __shared__ uint4 padl[4][64];   // each lane's padding block 0 (kept out of VGPRs)
    const int lane = threadIdx.x & 63;
    const uint32_t pl = lane & (kZcPieces - 1);  // the piece this lane hashes (lanes 32-63 mirror 0-31)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t g0 = blockIdx.x * kZcPieces;
    const uint32_t j = g0 + pl;
    const uint32_t jj = j < n ? j : n - 1;
    const uint32_t len = lens[jj];
    const uint32_t nfull = len >> 6;
    const uint32_t rem = len & 63u;
    const uint32_t nb = nfull + (rem <= 55 ? 1u : 2u);
    const uint32_t nb_wave = __builtin_amdgcn_readfirstlane(wave_max(nb));
    const uint32_t c16 = lane & 15;
    const uint32_t ntiles = (nb_wave + kZcTileBlocks - 1) / kZcTileBlocks;

    // Two register tiles in flight (32 KiB per wave; a third measured no
    // faster, profiles/r03/zero_copy/ab_async_t3.jsonl) and two LDS stage
    // buffers.  While the pair hashes tile t out of stage[t & 1], block bb
    // writes instructions 2bb, 2bb+1 of tile t+1 (landed in REG) into
    // stage[(t+1) & 1] and reloads them with tile t+3, so every block carries
    // the same 2 loads and 2 stage writes (staging a whole tile at its first
    // block made that block the pair's bound).  Plain arrays and the tile body
    // written out per register set: as a loop over a ring[2][16], or through a
    // lambda taking the tile by reference, hipcc kept the tiles in scratch.
    // LOADS: stage and reload; HASH: expand block b from stage[RD].  SEL = 0
    // for a tile whose blocks are all data for every lane (no per-lane select:
    // if-converted, the select and its padding reads cost 38 instructions in
    // EVERY block, profiles/r03/zero_copy/chain_probe.jsonl).
#define VX_ZC_TILE(REG, T, RD, SEL, LOADS, HASH)                                                        \
    {                                                                                                   \
        const uint32_t t = (T);                                                                         \
        _Pragma("unroll") for (uint32_t bb = 0; bb < kZcTileBlocks; ++bb) {                             \
            if (LOADS) {                                                                                \
                _Pragma("unroll") for (int k = 2 * bb; k < 2 * (int)bb + 2; ++k) {                      \
                    const uint32_t p = 4 * (k & 7) + (lane >> 4), c = c16 + 16 * (k >> 3);              \
                    stage[1 - (RD)][c][p] = REG[k];                                                     \
                }                                                                                       \
                zc_load_pair(REG, 2 * bb, zb, zl, t + 3);                                               \
            }                                                                                           \
            const uint32_t b = kZcTileBlocks * t + bb;                                                  \
            if ((HASH) && b < nb_wave) { /* wave-uniform */                                             \
                const uint4 q0 = stage[RD][4 * bb + 0][pl];                                           \
                const uint4 q1 = stage[RD][4 * bb + 1][pl];                                           \
                const uint4 q2 = stage[RD][4 * bb + 2][pl];                                           \
                const uint4 q3 = stage[RD][4 * bb + 3][pl];                                           \
                le_words(w, q0, q1, q2, q3);                                                            \
                if (SEL) {                                                                              \
                    const uint4 p0 = padl[0][lane], p1 = padl[1][lane], p2 = padl[2][lane], p3 = padl[3][lane]; \
                    const uint32_t pw[16] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w,            \
                                             p2.x, p2.y, p2.z, p2.w, p3.x, p3.y, p3.z, p3.w};           \
                    const bool is_pad0 = b == nfull;                                                    \
                    const bool is_pad1 = b == nfull + 1;                                                \
                    _Pragma("unroll") for (int k = 0; k < 16; ++k) {                                    \
                        uint32_t v = b < nfull ? w[k] : 0u;                                             \
                        v = is_pad0 ? pw[k] : v;                                                        \
                        if (k >= 14) v = (is_pad1 && rem > 55) ? (k == 14 ? bits_hi : bits_lo) : v;     \
                        w[k] = v;                                                                       \
                    }                                                                                   \
                }                                                                                       \
                expand_store(w, lds.w[ring_slot<S>(b)], lane);                                          \
            }                                                                                           \
            /* lgkmcnt(0) + s_barrier: this block's stage reads and writes are done before either */   \
            /* buffer is touched again (the consumer passes one barrier per block it hashes) */        \
            if (b < nb_wave) publish<S>(b);                                                             \
        }                                                                                               \
    }
    // Straight-line trips (tiles past the data load the zero line, blocks past
    // nb_wave are skipped), so the waitcnt pass sees the same 32 loads in
    // flight at the back edge as at the entry and waits for exactly the 2 it
    // stages next; a tile takes the select form only from the wave's first
    // block that is not data for all lanes.
    if (wave == 0) {
        // ---------------- consumer ----------------
        const uint32_t b1 = __builtin_amdgcn_readfirstlane(wave_min(nb));
        State s = iv();
        if (kLoader) __syncthreads();  // tile 0 staged
        consume<S, true>(s, lds, lane, nb_wave, b1, nb);
        if (lane < (int)kZcPieces && j < n) emit(s, j, digests, expected, matched, exp_index);
    } else if (kLoader && wave == 2) {
        // ---------------- loader ----------------
        uint64_t zb[8];
        uint32_t zl[8];
        uint4 ra[16], rb[16];
        uint32_t w[16];
        const uint32_t bits_hi = 0, bits_lo = 0;
        zc_setup(zb, zl, ra, rb, stage, srcs, lens, n, g0, lane);
        __syncthreads();
        for (uint32_t t0 = 0; t0 < ntiles; t0 += 2) {
            VX_ZC_TILE(rb, t0, 0, 0, 1, 0)
            VX_ZC_TILE(ra, t0 + 1, 1, 0, 1, 0)
        }
        (void)w;
        (void)bits_hi;
        (void)bits_lo;
        producer_done<S>(nb_wave);
    } else {
        // ---------------- producer ----------------
        // this lane's padding block 0 (its own tail bytes, read once)
        uint32_t padw[16];
        const uint8_t* q = reinterpret_cast<const uint8_t*>(srcs[jj]) + (size_t)nfull * 64;
        tail_words(padw, q, rem);
        const uint32_t bits_hi = (uint32_t)(((uint64_t)len * 8u) >> 32);
        const uint32_t bits_lo = (uint32_t)((uint64_t)len * 8u);
        if (rem <= 55) {
            padw[14] = bits_hi;
            padw[15] = bits_lo;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) padl[k][lane] = make_uint4(padw[4 * k], padw[4 * k + 1], padw[4 * k + 2], padw[4 * k + 3]);
        // The wave's first block that is not data for every lane: blocks
        // before it need no select (and no padding words).
        const uint32_t b_sel = __builtin_amdgcn_readfirstlane(wave_min(nfull));
        uint64_t zb[8];
        uint32_t zl[8];
        uint4 ra[16], rb[16];
        uint32_t w[16];
        if (kLoader)
            __syncthreads();
        else
            zc_setup(zb, zl, ra, rb, stage, srcs, lens, n, g0, lane);
        for (uint32_t t0 = 0; t0 < ntiles; t0 += 2) {
            if (kZcTileBlocks * (t0 + 1) <= b_sel) VX_ZC_TILE(rb, t0, 0, 0, !kLoader, 1) else VX_ZC_TILE(rb, t0, 0, 1, !kLoader, 1)
            if (kZcTileBlocks * (t0 + 2) <= b_sel) VX_ZC_TILE(ra, t0 + 1, 1, 0, !kLoader, 1) else VX_ZC_TILE(ra, t0 + 1, 1, 1, !kLoader, 1)
        }
        producer_done<S>(nb_wave);
    }
#undef VX_ZC_TILE
}

hipError_t launch_zero_copy(const uint64_t* srcs, const uint32_t* lens, uint32_t n, uint8_t* digests,
                            const uint8_t* expected, uint8_t* matched, bool loader, hipStream_t stream,
                            const uint32_t* exp_index) {
    if (n == 0) return hipSuccess;
    const uint32_t blocks = (n + kZcPieces - 1) / kZcPieces;
    if (loader)
        hipLaunchKernelGGL((sha1_zc_split_kernel<kSplitSlots, true>), dim3(blocks), dim3(3 * 64), 0, stream, srcs,
                           lens, n, digests, expected, matched, exp_index);
    else
        hipLaunchKernelGGL((sha1_zc_split_kernel<kSplitSlots, false>), dim3(blocks), dim3(kPairBlock), 0, stream,
                           srcs, lens, n, digests, expected, matched, exp_index);
    return hipGetLastError();
}

template <int R, bool kAlias = false, bool kFence = false>
hipError_t launch_uniform_lane_r(const uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint8_t* digests,
                                 const uint8_t* expected, uint8_t* matched, hipStream_t stream,
                                 const uint32_t* exp_index) {
    const uint32_t blocks = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL((sha1_uniform_kernel<R, kAlias, kFence>), dim3(blocks), dim3(kBlock), 0, stream, base, stride, len, n, digests,
                       expected, matched, exp_index);
    return hipGetLastError();
}

hipError_t launch_uniform_lane(const uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint8_t* digests,
                               const uint8_t* expected, uint8_t* matched, hipStream_t stream,
                               const uint32_t* exp_index) {
    // 4-deep fenced ring: measured 2.2 % fewer cycles per VALU than the
    // unfenced 3-deep ring (wait share 6.6 % -> 4.5 %).
    return launch_uniform_lane_r<kLaneRing, false, true>(base, stride, len, n, digests, expected, matched, stream,
                                                         exp_index);
}

hipError_t launch_ragged_lane(const uint8_t* base, const uint64_t* offsets, const uint32_t* lens,
                              const uint32_t* order, uint32_t n, uint8_t* digests, const uint8_t* expected,
                              uint8_t* matched, hipStream_t stream, const uint32_t* exp_index) {
    const uint32_t blocks = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(sha1_ragged_kernel, dim3(blocks), dim3(kBlock), 0, stream, base, offsets, lens, order, n,
                       digests, expected, matched, exp_index);
    return hipGetLastError();
}

}  // namespace vx

namespace vx {
hipError_t launch_uniform(const uint8_t* base, uint64_t stride, uint32_t len, uint32_t n, uint8_t* digests,
                          const uint8_t* expected, uint8_t* matched, hipStream_t stream, int variant,
                          const uint32_t* exp_index) {
    if (variant == kUniformLane) return launch_uniform_lane(base, stride, len, n, digests, expected, matched, stream, exp_index);
    if (variant == kUniformSplit) return launch_uniform_split(base, stride, len, n, digests, expected, matched, stream, exp_index);
    if (variant == kSplitRing2)
        return launch_uniform_split_s<2>(base, stride, len, n, digests, expected, matched, stream, exp_index);
    if (variant == kSplitRing3)
        return launch_uniform_split_s<3>(base, stride, len, n, digests, expected, matched, stream, exp_index);
    // Default: the integer VALU is the roofline once every SIMD has a wave
    // (n >= 65,536 with the lane kernel), and the split kernel's extra LDS
    // hand-off only costs there.  Below kSplitMaxPieces the chip has idle
    // SIMDs and the split kernel's shorter per-wave chain (405 vs 613 VALU per
    // block) finishes each piece sooner (DESIGN.md "Kernels", measured).
    if (n <= kSplitMaxPieces) return launch_uniform_split(base, stride, len, n, digests, expected, matched, stream, exp_index);
    return launch_uniform_lane(base, stride, len, n, digests, expected, matched, stream, exp_index);
}
}  // namespace vx

namespace vx {
// Kernel choice for a ragged batch from its longest piece and total bytes
// (DESIGN.md §3.4).  Each kernel's time is bounded below by its throughput
// over all bytes and by the longest piece's chain, whichever is larger:
//   lane : max(total / 3.4 TB/s, blocks(max_len) x 1.18 us)
//   split: max(total / 2.5 TB/s, blocks(max_len) x 0.77 us)
// (config 2 and config 3 measurements, §3.5: the lane kernel's VALU-bound
// rate and per-block chain, the split kernel's; 0.87 us before the asm
// consumer of §3.2.1).  Config 3's 4 MiB pieces make
// it chain-bound: 77 ms lane vs 57 ms split, though it has 283,648 pieces.
//
// Split batches whose whole-chip work at HALF the split throughput (one pair
// per CU) is still at most half their longest chain run wide (kSplitWide).
int plan_ragged(uint32_t n, uint64_t max_len, uint64_t total_len) {
    (void)n;
    const double blocks = (double)((max_len + 9 + 63) / 64);
    const double lane = std::max((double)total_len / 3.4e12, blocks * 1.18e-6);
    const double split = std::max((double)total_len / 2.5e12, blocks * 0.77e-6);
    if (lane < split) return kUniformLane;
    return (double)total_len / 1.25e12 <= 0.5 * blocks * 0.77e-6 ? kSplitWide : kUniformSplit;
}

// variant 0 without a plan: the split kernel.  A batch whose lengths really
// differ is usually bound by its longest chain, where split's shorter per-block
// chain wins by up to 2.3x; the lane kernel is at most 1.4x faster, and only on
// throughput-bound batches of near-equal pieces (use the uniform entry, or
// vx_sha1_device_ragged_hint, for those).
hipError_t launch_ragged(const uint8_t* base, const uint64_t* offsets, const uint32_t* lens, const uint32_t* order,
                         uint32_t n, uint8_t* digests, const uint8_t* expected, uint8_t* matched,
                         hipStream_t stream, int variant, const uint32_t* exp_index) {
    if (variant == kUniformLane) return launch_ragged_lane(base, offsets, lens, order, n, digests, expected, matched, stream, exp_index);
    if (variant == kSplitRing2)
        return launch_ragged_split_s<2>(base, offsets, lens, order, n, digests, expected, matched, stream, exp_index);
    if (variant == kSplitRing3)
        return launch_ragged_split_s<3>(base, offsets, lens, order, n, digests, expected, matched, stream, exp_index);
    if (variant == kSplitWide)
        return launch_ragged_split_s<kSplitSlots>(base, offsets, lens, order, n, digests, expected, matched, stream,
                                                  exp_index, true);
    return launch_ragged_split(base, offsets, lens, order, n, digests, expected, matched, stream, exp_index);
}
}  // namespace vx
