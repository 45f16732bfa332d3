// pair_probe.hip — what costs the split kernel's consumer its last ~10 %?
//
// The generated consumer (vortex_amd/csrc/sha1_consumer_asm.inc) runs a block
// in ~1,650 cycles alone (tools/native/rounds_sched_probe.hip) but ~1,850 in
// the kernels.  This pairs it with a synthetic producer wave on the real
// ring protocol (3 LDS slots, one barrier per block, RingLds layout) and
// switches the producer's work on and off:
//   0  producer passes the barriers only
//   1  + writes each block's 20 x ds_write_b128 into its slot (as expand_store)
//   2  + ~210 VALU per block (the schedule's load: 16 perm + 192 + stores' data)
//   3  as 2, two pairs per CU (the kernels' occupancy with 60 KiB per pair)
//   4  as 2 with the producer's VALU as a rolled loop (little instruction fetch)
//   5  as 2 with the consumer at s_setprio 3
//   6  as 2 with a 6-slot ring and one barrier per PAIR of blocks (120 KiB LDS)
//   7  as 2 with no barriers: an LDS flag handshake (producer count / consumer
//      count, tools/gen_sha1_rounds.py consumer_flags_asm), bounded waits
//   8  as 7 with the producer passing the flags only (no LDS writes, no VALU)
//   9  as 2 with the producer's 210 VALU all VOP2 (v_add_u32_e32): does the
//      interference follow the producer's instruction count or its VALU cycles?
//   10 as 2 with half the producer VALU (105 VOP3)
//   11 as 1 (LDS writes, no VALU) with the 6-slot ring: one barrier per 2 blocks
//   12 the real producer's VALU: 16 v_perm + 64 x (xor3, xor, rotl1) as VOP3
//      (bitop3 0x96, bitop3 0x3c, alignbit), 3-slot ring
//   13 as 12 with the 6-slot ring
//   14 as 12 with the 2-input xor as VOP2 v_xor_b32_e32 (144 VOP3 + 64 VOP2)
//   15 as 14 with the 6-slot ring
//   16 no synchronisation: the consumer with s_barrier -> s_nop 0 and an idle
//      producer wave (what the barriers cost; the consumer reads stale slots)
//   17 as 16 with the producer wave running the real producer's VALU unsynchronised
//   18-22 as 16 with the next block's 20 ring reads placed differently: none (the
//      loop's rounds-only floor), 2 bursts of 10 (rounds 0, 40), 4 of 5 (rounds 0,
//      20, 40, 60), one read every 4 rounds, all 20 at round 60
// The consumer stamps s_memtime around its whole loop; prints cycles per
// block (median over pairs) and the wall ns per block.  No HBM traffic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "../../vortex_amd/csrc/sha1_consumer_asm.inc"
#include "sha1_consumer6_asm.inc"  // python tools/gen_sha1_rounds.py --consumer6 tools/native/sha1_consumer6_asm.inc
#include "sha1_consumerf_asm.inc"  // python tools/gen_sha1_rounds.py --consumerf tools/native/sha1_consumerf_asm.inc
#include "sha1_consumernb_asm.inc"  // python tools/gen_sha1_rounds.py --consumer-nobarrier tools/native/sha1_consumernb_asm.inc
#include "sha1_consumer_place_asm.inc"  // python tools/gen_sha1_rounds.py --consumer-placements tools/native/sha1_consumer_place_asm.inc

template <int S>
struct Ring {
    uint4 w[S][20][64];
};

template <int P>
__global__ __launch_bounds__(128) void pair(uint32_t nb, uint32_t* out, unsigned long long* cyc) {
    constexpr int S = (P == 6 || P == 11 || P == 13 || P == 15) ? 6 : 3;  // 6: barrier per 2 blocks (VX_CONSUMER6_ASM)
    __shared__ Ring<S> lds;
    __shared__ uint32_t flags[4];  // P = 7, 8: {prod, cons, consumer gave up, producer gave up}
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr bool F = P == 7 || P == 8;  // flag handshake instead of barriers
    if (F) {
        if (threadIdx.x < 4) flags[threadIdx.x] = 0;
        __syncthreads();
    }
    if (wave == 1 && F) {  // flag-handshake producer
        uint32_t x = lane * 0x9E3779B9u, y = 0x12345u + lane;
        for (uint32_t b = 0; b < nb; ++b) {
            if (P == 7) {
#pragma unroll
                for (int i = 0; i < 70; ++i) {  // 210 VALU
                    x = __builtin_amdgcn_alignbit(x, x, 31) ^ y;
                    y = __builtin_amdgcn_bitop3_b32(x, y, 0x5a5a5a5au, 0x96);
                    x = x + y;
                }
            }
            uint32_t polls = 0;  // slot b % 3 is free once the consumer has read block b - 3
            while ((int)__hip_atomic_load(&flags[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < (int)b - 2) {
                __builtin_amdgcn_s_sleep(1);
                if (++polls > (1u << 22)) {
                    flags[3] = 1;
                    break;
                }
            }
            if (P == 7) {
#pragma unroll
                for (int q = 0; q < 20; ++q) lds.w[b % S][q][lane] = make_uint4(x + q, y, x ^ q, b);
            }
            __hip_atomic_store(&flags[0], b + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        out[blockIdx.x * 64 + lane] = x ^ y;
        return;
    }
    if (wave == 1 && P >= 16) {  // unsynchronised producer
        if (P == 17) {
            uint32_t w[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) w[k] = lane * 0x9E3779B9u + k;
            for (uint32_t b = 0; b < nb; ++b) {
#pragma unroll
                for (int k = 0; k < 16; ++k) w[k] = __builtin_amdgcn_perm(w[k], w[k] + b, 0x00010203u);
#pragma unroll
                for (int t = 16; t < 80; ++t) {
                    uint32_t v = __builtin_amdgcn_bitop3_b32(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15], 0x96);
                    v = __builtin_amdgcn_bitop3_b32(v, w[t & 15], w[t & 15], 0x3C);
                    w[t & 15] = __builtin_amdgcn_alignbit(v, v, 31);
                }
#pragma unroll
                for (int q = 0; q < 20; ++q)
                    lds.w[b % S][q][lane] = make_uint4(w[(4 * q) & 15], w[(4 * q + 1) & 15], w[(4 * q + 2) & 15],
                                                       w[(4 * q + 3) & 15]);
            }
            out[blockIdx.x * 64 + lane] = w[0];
        }
        return;
    }
    if (wave == 1) {  // producer
        uint32_t x = lane * 0x9E3779B9u, y = 0x12345u + lane;
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = x + k * y;
        for (uint32_t b = 0; b < nb; ++b) {
            if (P >= 12) {  // the real producer's schedule work per block
#pragma unroll
                for (int k = 0; k < 16; ++k) w[k] = __builtin_amdgcn_perm(w[k], w[k] + b, 0x00010203u);
#pragma unroll
                for (int t = 16; t < 80; ++t) {
                    uint32_t v = __builtin_amdgcn_bitop3_b32(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15], 0x96);
                    v = (P >= 14) ? (v ^ w[t & 15]) : __builtin_amdgcn_bitop3_b32(v, w[t & 15], w[t & 15], 0x3C);
                    w[t & 15] = __builtin_amdgcn_alignbit(v, v, 31);
                }
                x = w[0];
                y = w[5];
            } else if (P == 4) {
                // the same 210 VALU as a short rolled loop (no instruction-fetch stream)
                for (int i = 0; i < 70; ++i) {
                    x = __builtin_amdgcn_alignbit(x, x, 31) ^ y;
                    y = __builtin_amdgcn_bitop3_b32(x, y, 0x5a5a5a5au, 0x96);
                    x = x + y;
                    asm volatile("" : "+v"(x), "+v"(y));
                }
            } else if (P == 9) {
#pragma unroll
                for (int i = 0; i < 105; ++i) {  // 210 VOP2 adds
                    x = x + y;
                    y = y + x;
                }
            } else if (P == 10) {
#pragma unroll
                for (int i = 0; i < 35; ++i) {  // 105 VALU
                    x = __builtin_amdgcn_alignbit(x, x, 31) ^ y;
                    y = __builtin_amdgcn_bitop3_b32(x, y, 0x5a5a5a5au, 0x96);
                    x = x + y;
                }
            } else if (P >= 2) {
#pragma unroll
                for (int i = 0; i < 70; ++i) {  // 210 VALU
                    x = __builtin_amdgcn_alignbit(x, x, 31) ^ y;
                    y = __builtin_amdgcn_bitop3_b32(x, y, 0x5a5a5a5au, 0x96);
                    x = x + y;
                }
            }
            if (P >= 12) {
#pragma unroll
                for (int q = 0; q < 20; ++q)
                    lds.w[b % S][q][lane] = make_uint4(w[(4 * q) & 15], w[(4 * q + 1) & 15], w[(4 * q + 2) & 15],
                                                       w[(4 * q + 3) & 15]);
            } else if (P >= 1) {
#pragma unroll
                for (int q = 0; q < 20; ++q) lds.w[b % S][q][lane] = make_uint4(x + q, y, x ^ q, b);
            }
            if (S == 3 ? b >= 1 : ((b & 1) || b + 1 == nb) && b >= 2) __syncthreads();
        }
        if (nb) {
            __syncthreads();
            __syncthreads();
        }
        out[blockIdx.x * 64 + lane] = x ^ y;
        return;
    }
    if (P == 5) __builtin_amdgcn_s_setprio(3);
    uint32_t h0 = 0x67452301u + lane, h1 = 0xEFCDAB89u, h2 = 0x98BADCFEu, h3 = 0x10325476u, h4 = 0xC3D2E1F0u;
    const uint32_t addr = (uint32_t)(uintptr_t)&lds.w[0][0][lane];
    const uint32_t addr3 = (uint32_t)(uintptr_t)&lds.w[S == 6 ? 3 : 0][0][lane];
    const uint32_t zero = 0;
    const uint32_t faddr = (uint32_t)(uintptr_t)&flags[0];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#define VX_NB(M)                                                                    \
    asm volatile(M : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "+v"(h4)             \
                 : "v"(addr), "s"(nb), "s"(nb), "v"(zero)                          \
                 : VX_CONSUMER_ASM_CLOBBERS, "memory")
    if (P == 18) VX_NB(VX_CONSUMERNB_NONE_ASM);
    else if (P == 19) VX_NB(VX_CONSUMERNB_SPLIT2_ASM);
    else if (P == 20) VX_NB(VX_CONSUMERNB_SPLIT4_ASM);
    else if (P == 21) VX_NB(VX_CONSUMERNB_SPREAD4_ASM);
    else if (P == 22) VX_NB(VX_CONSUMERNB_LATE_ASM);
    else if (P >= 16)
        asm volatile(VX_CONSUMERNB_ASM
                     : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "+v"(h4)
                     : "v"(addr), "s"(nb), "s"(nb), "v"(zero)
                     : VX_CONSUMER_ASM_CLOBBERS, "memory");
    else if (F)
        asm volatile(VX_CONSUMERF_ASM
                     : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "+v"(h4)
                     : "v"(addr), "s"(nb), "s"(nb), "v"(zero), "v"(faddr)
                     : VX_CONSUMERF_ASM_CLOBBERS, "memory");
    else if (S == 6)
        asm volatile(VX_CONSUMER6_ASM
                     : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "+v"(h4)
                     : "v"(addr), "s"(nb), "s"(nb), "v"(zero), "v"(addr3)
                     : VX_CONSUMER6_ASM_CLOBBERS, "memory");
    else
        asm volatile(VX_CONSUMER_ASM
                     : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "+v"(h4)
                     : "v"(addr), "s"(nb), "s"(nb), "v"(zero)
                     : VX_CONSUMER_ASM_CLOBBERS, "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + lane] = h0 ^ h1 ^ h2 ^ h3 ^ h4;
    if (lane == 0) cyc[blockIdx.x] = (F && (flags[2] | flags[3])) ? ~0ull : t1 - t0;
}

template <int P>
static void run(const char* name, int grid, uint32_t* d, unsigned long long* dc, bool comma) {
    const uint32_t nb = 20000;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(pair<P>, dim3(grid), dim3(128), 0, 0, 500u, d, dc);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(pair<P>, dim3(grid), dim3(128), 0, 0, nb, d, dc);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    std::vector<unsigned long long> c(grid);
    (void)hipMemcpy(c.data(), dc, grid * 8, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    if (c.back() == ~0ull) std::printf("%s\"%s_GAVE_UP\": 1", comma ? ", " : "", name);
    std::printf("%s\"%s\": {\"cycles_per_block\": %.1f, \"ns_per_block\": %.1f, \"pairs\": %d}", comma ? ", " : "",
                name, (double)c[grid / 2] / nb, ms * 1e6 / nb, grid);
}

int main() {
    uint32_t* d = nullptr;
    unsigned long long* dc = nullptr;
    if (hipMalloc(&d, 512 * 64 * 4) != hipSuccess || hipMalloc(&dc, 512 * 8) != hipSuccess) return 1;
    std::printf("{");
    run<0>("barriers_only", 64, d, dc, false);
    run<1>("lds_writes", 64, d, dc, true);
    run<2>("lds_writes_valu", 64, d, dc, true);
    run<2>("lds_writes_valu_2_pairs_per_cu", 512, d, dc, true);
    run<4>("lds_writes_valu_rolled_loop", 64, d, dc, true);
    run<5>("lds_writes_valu_consumer_prio3", 64, d, dc, true);
    run<6>("lds_writes_valu_6slots_barrier_per_pair", 64, d, dc, true);
    run<8>("flags_only", 64, d, dc, true);
    run<7>("flags_lds_writes_valu", 64, d, dc, true);
    run<7>("flags_lds_writes_valu_2_pairs_per_cu", 512, d, dc, true);
    run<9>("lds_writes_valu_vop2_adds", 64, d, dc, true);
    run<10>("lds_writes_half_valu", 64, d, dc, true);
    run<11>("lds_writes_6slots", 64, d, dc, true);
    run<12>("real_producer_vop3_xor", 64, d, dc, true);
    run<13>("real_producer_vop3_xor_6slots", 64, d, dc, true);
    run<14>("real_producer_vop2_xor", 64, d, dc, true);
    run<15>("real_producer_vop2_xor_6slots", 64, d, dc, true);
    run<12>("real_producer_vop3_xor_2_pairs_per_cu", 512, d, dc, true);
    run<14>("real_producer_vop2_xor_2_pairs_per_cu", 512, d, dc, true);
    run<16>("no_barriers_idle_producer", 64, d, dc, true);
    run<17>("no_barriers_real_producer_unsynced", 64, d, dc, true);
    run<18>("no_barriers_reads_none", 64, d, dc, true);
    run<19>("no_barriers_reads_split2", 64, d, dc, true);
    run<20>("no_barriers_reads_split4", 64, d, dc, true);
    run<21>("no_barriers_reads_spread4", 64, d, dc, true);
    run<22>("no_barriers_reads_late", 64, d, dc, true);
    std::printf("}\n");
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
