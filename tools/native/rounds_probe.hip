// rounds_probe.hip — what does one wave's SHA-1 block cost when the wave
// does nothing but the 80 rounds (the split kernel's consumer, DESIGN.md
// §3.2)?  16 workgroups (far below the power cap), NB blocks per lane, words
// from registers; three variants:
//   0  rounds only (words in registers; an empty asm per block stops the
//      compiler from hoisting anything across blocks)
//   1  + the next block's 20 ds_read_b128 from LDS, issued before the rounds
//      (the consumer's burst)
//   2  + one s_barrier per block with a second wave that only waits
// Prints ns per block and, at the clock given as argv[1] (GHz, e.g. 2.4),
// cycles per block and per instruction (425 rounds+feed-forward VALU).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../../vortex_amd/csrc/sha1_device.hpp"

using vx::State;

__device__ __forceinline__ void rounds(State& s, const uint4 (&w)[20]) {
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
                k = 0x5A827999u;
            } else if (t < 40) {
                f = VX_PAR(b, c, d);
                k = 0x6ED9EBA1u;
            } else if (t < 60) {
                f = VX_MAJ(b, c, d);
                k = 0x8F1BBCDCu;
            } else {
                f = VX_PAR(b, c, d);
                k = 0xCA62C1D6u;
            }
#ifdef VX_ROUND_X
            uint32_t x = e + k + wq[j];
            asm("" : "+v"(x));  // keep LLVM from reassociating: a' = add3(rotl5(a), f, x)
            const uint32_t tmp = vx::rotl(a, 5) + f + x;
#else
            const uint32_t tmp = vx::rotl(a, 5) + f + e + k + wq[j];
#endif
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
__global__ __launch_bounds__(128) void probe(uint32_t nb, uint32_t* out) {
    __shared__ uint4 ring[20][64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    for (int q = 0; q < 20; ++q) ring[q][lane] = make_uint4(q, lane, q * lane, 7);
    __syncthreads();
    if (wave == 1) {  // partner: passes the same barriers, nothing else
        if (V == 2)
            for (uint32_t b = 0; b < nb; b += 2) {
                __syncthreads();
                __syncthreads();
            }
        return;
    }
    State s{0x67452301u + lane, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    uint4 w0[20], w1[20];
    for (int q = 0; q < 20; ++q) w0[q] = w1[q] = ring[q][lane];
    __builtin_amdgcn_s_waitcnt(0xC07F);  // drained before the loop, as the consumer
    // As the consumer: two register sets, the next block's reads issued
    // before this block's rounds, lgkmcnt(0) (+ barrier) at the block's end,
    // every block's rounds 8-byte aligned.
    auto block = [&](uint4 (&cur)[20], uint4 (&nxt)[20]) {
        if (V >= 1) {
#pragma unroll
            for (int q = 0; q < 20; ++q) nxt[q] = ring[q][lane];
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile(".p2align 3");
        __builtin_amdgcn_sched_barrier(0);
        rounds(s, cur);
        asm volatile("" : "+v"(s.h0), "+v"(s.h1), "+v"(s.h2), "+v"(s.h3), "+v"(s.h4));
        if (V == 0) {
#pragma unroll
            for (int q = 0; q < 20; ++q)
                asm volatile("" : "+v"(cur[q].x), "+v"(cur[q].y), "+v"(cur[q].z), "+v"(cur[q].w));
        }
        __builtin_amdgcn_sched_barrier(0);
        if (V >= 1) __builtin_amdgcn_s_waitcnt(0xC07F);
        if (V == 2) __syncthreads();
    };
    for (uint32_t b = 0; b < nb; b += 2) {
        block(w0, w1);
        block(w1, w0);
    }
    out[blockIdx.x * 64 + lane] = s.h0 ^ s.h1 ^ s.h2 ^ s.h3 ^ s.h4;
}

template <int V>
static float run(uint32_t nb, uint32_t* d) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(probe<V>, dim3(16), dim3(128), 0, 0, 1000u, d);  // warm
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(probe<V>, dim3(16), dim3(128), 0, 0, nb, d);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main(int argc, char** argv) {
    const double ghz = argc > 1 ? std::atof(argv[1]) : 2.4;
    const uint32_t nb = 200000;
    uint32_t* d = nullptr;
    if (hipMalloc(&d, 16 * 64 * 4) != hipSuccess) return 1;
    std::printf("{\"blocks\": %u, \"assumed_GHz\": %.2f", nb, ghz);
    const char* names[3] = {"rounds_only", "plus_lds_reads", "plus_barrier"};
    for (int v = 0; v < 3; ++v) {
        const float ms = v == 0 ? run<0>(nb, d) : v == 1 ? run<1>(nb, d) : run<2>(nb, d);
        const double ns = ms * 1e6 / nb;
        std::printf(", \"%s\": {\"ns_per_block\": %.1f, \"cycles_per_block\": %.0f, \"cycles_per_valu\": %.3f}",
                    names[v], ns, ns * ghz, ns * ghz / 405.0);
    }
    std::printf("}\n");
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
