// rounds_sched_probe.hip — does the ORDER of a SHA-1 round's five VALU ops
// limit a lone wave (the split kernel's consumer)?
//
// The consumer issues 405 VALU per block at one wave per SIMD, i.e. at most
// one instruction per 4 cycles, and a rounds-only wave measured 4.3-4.6
// cycles per instruction (profiles/r01/valu/rounds_probe*.json).  A round has
// a dependency chain of depth 2 (a' = add3(rotl5(a), f(a, c, d), x)) and
// three ops off the chain; if a dependent op issued right behind its producer
// stalls, the order decides whether the fillers hide it.  Variants, words in
// registers, 16 workgroups (far below the power cap):
//   0  hipcc's schedule of the kernel's round code (rounds_regs)
//   1  hand-ordered stream X(t+1), rotl5(a), f, rotl30(a), add3 -> a': every
//      dependent pair at least 2 issue slots apart (inline asm, volatile)
//   2  hand-ordered naive stream rotl5, f, X(t), add3, rotl30: the add3 right
//      behind f, rotl5 of the new a right behind its add3
//   3  as 1, plus the next block's 20 ds_read_b128 in a burst (the consumer)
//   4  the order of 1 with builtins, fenced op by op (no asm nops)
//   5  as 4, plus the consumer's ds_read burst
//   6  tools/gen_sha1_rounds.py's stream on fixed registers, one asm per block
//      (the words are whatever v100-v179 hold: timing only)
//   7  as 6, plus the consumer's ds_read burst
// Each wave stamps s_memtime around its loop; prints cycles per block and
// per VALU (405 per block) as the median over waves, and the wall ns/block.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../vortex_amd/csrc/sha1_device.hpp"
#include "sha1_rounds_fixed.inc"

using vx::State;

__device__ __forceinline__ uint32_t r5(uint32_t a) {
    uint32_t r;
    asm volatile("v_alignbit_b32 %0, %1, %1, 27" : "=v"(r) : "v"(a));
    return r;
}
__device__ __forceinline__ uint32_t r30(uint32_t a) {
    uint32_t r;
    asm volatile("v_alignbit_b32 %0, %1, %1, 2" : "=v"(r) : "v"(a));
    return r;
}
template <int T>
__device__ __forceinline__ uint32_t ff(uint32_t b, uint32_t c, uint32_t d) {
    uint32_t r;
    if (T < 20)
        asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "v"(b), "v"(c), "v"(d));
    else if (T < 40 || T >= 60)
        asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(b), "v"(c), "v"(d));
    else
        asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe8" : "=v"(r) : "v"(b), "v"(c), "v"(d));
    return r;
}
__device__ __forceinline__ uint32_t add3v(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t add3k(uint32_t e, uint32_t k, uint32_t w) {
    uint32_t r;
    asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(e), "s"(k), "v"(w));
    return r;
}
__host__ __device__ constexpr uint32_t kof(int t) {
    return t < 20 ? 0x5A827999u : t < 40 ? 0x6ED9EBA1u : t < 60 ? 0x8F1BBCDCu : 0xCA62C1D6u;
}

// A_t = a after round t (A_{-1} = h0, A_{-2} = h1); C_t = rotl30(A_{t-1}) is c
// of round t+1 (C_{-1} = h2, C_{-2} = h3, C_{-3} = h4), so round t uses
// b = A_{t-1}, c = C_{t-1}, d = C_{t-2}, e = C_{t-3}.
template <bool kPipelined>
__device__ __forceinline__ void rounds_asm(State& s, const uint4 (&w)[20]) {
    uint32_t W[80];
#pragma unroll
    for (int q = 0; q < 20; ++q) {
        W[4 * q] = w[q].x;
        W[4 * q + 1] = w[q].y;
        W[4 * q + 2] = w[q].z;
        W[4 * q + 3] = w[q].w;
    }
    uint32_t A[80], C[80], X[80];
    auto Aof = [&](int t) { return t >= 0 ? A[t] : (t == -1 ? s.h0 : s.h1); };
    auto Cof = [&](int t) { return t >= 0 ? C[t] : (t == -1 ? s.h2 : t == -2 ? s.h3 : s.h4); };
    if (kPipelined) X[0] = add3k(Cof(-3), kof(0), W[0]);
#pragma unroll
    for (int t = 0; t < 80; ++t) {
        if (kPipelined) {
            if (t + 1 < 80) X[t + 1] = add3k(Cof(t - 2), kof(t + 1), W[t + 1]);
            const uint32_t R = r5(Aof(t - 1));
            uint32_t F;
            if (t < 20) F = ff<0>(Aof(t - 1), Cof(t - 1), Cof(t - 2));
            else if (t < 40) F = ff<20>(Aof(t - 1), Cof(t - 1), Cof(t - 2));
            else if (t < 60) F = ff<40>(Aof(t - 1), Cof(t - 1), Cof(t - 2));
            else F = ff<60>(Aof(t - 1), Cof(t - 1), Cof(t - 2));
            C[t] = r30(Aof(t - 1));
            A[t] = add3v(R, F, X[t]);
        } else {
            const uint32_t R = r5(Aof(t - 1));
            uint32_t F;
            if (t < 20) F = ff<0>(Aof(t - 1), Cof(t - 1), Cof(t - 2));
            else if (t < 40) F = ff<20>(Aof(t - 1), Cof(t - 1), Cof(t - 2));
            else if (t < 60) F = ff<40>(Aof(t - 1), Cof(t - 1), Cof(t - 2));
            else F = ff<60>(Aof(t - 1), Cof(t - 1), Cof(t - 2));
            X[t] = add3k(Cof(t - 3), kof(t), W[t]);
            A[t] = add3v(R, F, X[t]);
            C[t] = r30(Aof(t - 1));
        }
    }
    s.h0 += A[79];
    s.h1 += A[78];
    s.h2 += C[79];
    s.h3 += C[78];
    s.h4 += C[77];
}

// The same pipelined order with builtins (no inline asm: hipcc puts an
// s_nop 0 behind every asm VALU op it cannot see into), each op fenced by
// sched_barrier(0) and each value pinned by an empty asm so LLVM neither
// reassociates the adds nor moves anything.
#define VX_PIN(x) asm volatile("" : "+v"(x))
#define VX_FENCE() __builtin_amdgcn_sched_barrier(0)
__device__ __forceinline__ void rounds_fenced(State& s, const uint4 (&w)[20]) {
    uint32_t W[80];
#pragma unroll
    for (int q = 0; q < 20; ++q) {
        W[4 * q] = w[q].x;
        W[4 * q + 1] = w[q].y;
        W[4 * q + 2] = w[q].z;
        W[4 * q + 3] = w[q].w;
    }
    uint32_t A[80], C[80], X[80];
    auto Aof = [&](int t) { return t >= 0 ? A[t] : (t == -1 ? s.h0 : s.h1); };
    auto Cof = [&](int t) { return t >= 0 ? C[t] : (t == -1 ? s.h2 : t == -2 ? s.h3 : s.h4); };
    X[0] = Cof(-3) + kof(0) + W[0];
    VX_PIN(X[0]);
#pragma unroll
    for (int t = 0; t < 80; ++t) {
        if (t + 1 < 80) {
            X[t + 1] = Cof(t - 2) + kof(t + 1) + W[t + 1];
            VX_PIN(X[t + 1]);
        }
        VX_FENCE();
        uint32_t R = vx::rotl(Aof(t - 1), 5);
        VX_PIN(R);
        VX_FENCE();
        uint32_t F;
        if (t < 20) F = VX_CH(Aof(t - 1), Cof(t - 1), Cof(t - 2));
        else if (t < 40 || t >= 60) F = VX_PAR(Aof(t - 1), Cof(t - 1), Cof(t - 2));
        else F = VX_MAJ(Aof(t - 1), Cof(t - 1), Cof(t - 2));
        VX_PIN(F);
        VX_FENCE();
        C[t] = vx::rotl(Aof(t - 1), 30);
        VX_PIN(C[t]);
        VX_FENCE();
        A[t] = R + F + X[t];
        VX_PIN(A[t]);
        VX_FENCE();
    }
    s.h0 += A[79];
    s.h1 += A[78];
    s.h2 += C[79];
    s.h3 += C[78];
    s.h4 += C[77];
}

__device__ __forceinline__ void rounds_cc(State& s, const uint4 (&w)[20]) {
    uint32_t a = s.h0, b = s.h1, c = s.h2, d = s.h3, e = s.h4;
#pragma unroll
    for (int q = 0; q < 20; ++q) {
        const uint32_t wq[4] = {w[q].x, w[q].y, w[q].z, w[q].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = 4 * q + j;
            uint32_t f;
            if (t < 20) f = VX_CH(b, c, d);
            else if (t < 40) f = VX_PAR(b, c, d);
            else if (t < 60) f = VX_MAJ(b, c, d);
            else f = VX_PAR(b, c, d);
            const uint32_t tmp = vx::rotl(a, 5) + f + e + kof(t) + wq[j];
            e = d;
            d = c;
            c = vx::rotl(b, 30);
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

template <int V>
__global__ __launch_bounds__(64) void probe(uint32_t nb, uint32_t* out, unsigned long long* cyc) {
    __shared__ uint4 ring[20][64];
    const int lane = threadIdx.x & 63;
    for (int q = 0; q < 20; ++q) ring[q][lane] = make_uint4(q, lane, q * lane, 7);
    __syncthreads();
    State s{0x67452301u + lane, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    uint4 w0[20], w1[20];
    for (int q = 0; q < 20; ++q) w0[q] = w1[q] = ring[q][lane];
    __builtin_amdgcn_s_waitcnt(0xC07F);
    auto block = [&](uint4 (&cur)[20], uint4 (&nxt)[20]) {
        if (V == 3 || V == 5 || V == 7) {
#pragma unroll
            for (int q = 0; q < 20; ++q) nxt[q] = ring[q][lane];
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile(".p2align 3");
        __builtin_amdgcn_sched_barrier(0);
        if (V == 6 || V == 7) asm volatile(VX_ROUNDS_FIXED ::: VX_ROUNDS_FIXED_CLOBBERS, "s20", "s21", "s22", "s23");
        else if (V == 0) rounds_cc(s, cur);
        else if (V == 2) rounds_asm<false>(s, cur);
        else if (V >= 4) rounds_fenced(s, cur);
        else rounds_asm<true>(s, cur);
        asm volatile("" : "+v"(s.h0), "+v"(s.h1), "+v"(s.h2), "+v"(s.h3), "+v"(s.h4));
        if (V != 3 && V != 5 && V != 7) {
#pragma unroll
            for (int q = 0; q < 20; ++q)
                asm volatile("" : "+v"(cur[q].x), "+v"(cur[q].y), "+v"(cur[q].z), "+v"(cur[q].w));
        }
        __builtin_amdgcn_sched_barrier(0);
        if (V == 3 || V == 5 || V == 7) __builtin_amdgcn_s_waitcnt(0xC07F);
    };
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t b = 0; b < nb; b += 2) {
        block(w0, w1);
        block(w1, w0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + lane] = s.h0 ^ s.h1 ^ s.h2 ^ s.h3 ^ s.h4;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
static void run(uint32_t nb, uint32_t* d, unsigned long long* dc, const char* name, bool comma) {
    const int G = 64;  // one wave per workgroup, 64 workgroups: far below the power cap
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(probe<V>, dim3(G), dim3(64), 0, 0, 2000u, d, dc);  // warm
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(probe<V>, dim3(G), dim3(64), 0, 0, nb, d, dc);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    std::vector<unsigned long long> c(G);
    (void)hipMemcpy(c.data(), dc, G * 8, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    const double cpb = (double)c[G / 2] / nb;
    std::printf("%s\"%s\": {\"ns_per_block\": %.1f, \"cycles_per_block\": %.1f, \"cycles_per_valu\": %.3f, "
                "\"clock_GHz\": %.3f}",
                comma ? ", " : "", name, ms * 1e6 / nb, cpb, cpb / 405.0, cpb / (ms * 1e6 / nb));
}

int main() {
    const uint32_t nb = 200000;
    uint32_t* d = nullptr;
    unsigned long long* dc = nullptr;
    if (hipMalloc(&d, 64 * 64 * 4) != hipSuccess || hipMalloc(&dc, 64 * 8) != hipSuccess) return 1;
    std::printf("{\"blocks\": %u, ", nb);
    run<0>(nb, d, dc, "compiler", false);
    run<1>(nb, d, dc, "asm_pipelined", true);
    run<2>(nb, d, dc, "asm_naive", true);
    run<3>(nb, d, dc, "asm_pipelined_lds_burst", true);
    run<4>(nb, d, dc, "fenced_pipelined", true);
    run<5>(nb, d, dc, "fenced_pipelined_lds_burst", true);
    run<6>(nb, d, dc, "fixed_regs", true);
    run<7>(nb, d, dc, "fixed_regs_lds_burst", true);
    std::printf("}\n");
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
