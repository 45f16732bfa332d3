// valu_probe.hip — issue rate of SHA-1's integer VALU ops on one gfx950 SIMD.
//
// MI355X_MICROARCH.md: a CDNA4 SIMD is 32 lanes wide, so a wave64 VALU op
// occupies it for 2 cycles, but one wave alone issues at most every ~4.  The
// SHA-1 kernels run v_alignbit_b32 / v_bitop3_b32 / v_add3_u32 / v_xor_b32.
// This measures cycles per instruction per wave (s_memtime, in-kernel) for a
// stream of independent such ops at 1, 2 and 4 waves per SIMD, on a few CUs
// only (so the chip stays far from its power cap and runs at full clock).
// If 2 waves/SIMD each still take ~4 cycles per op, the SIMD retires one
// wave64 integer op every 2 cycles (full rate); if ~8, every 4.
// Prints one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));        \
            return 1;                                                           \
        }                                                                       \
    } while (0)

constexpr int kChains = 8;
constexpr int kIter = 4096;

// 8 independent chains; per chain and iteration: alignbit, bitop3, add3, xor
// = 4 VALU, so 32 VALU per iteration with no dependency between neighbours.
template <int WGSIZE>
__global__ __launch_bounds__(WGSIZE) void valu_kernel(uint32_t seed, uint32_t* sink, uint64_t* cycles) {
    uint32_t x[kChains], y[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
        x[c] = seed * (c + 1) + threadIdx.x;
        y[c] = seed ^ (c * 0x9E3779B9u) ^ threadIdx.x;
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIter; ++it) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            uint32_t r = __builtin_amdgcn_alignbit(x[c], x[c], 27);
            uint32_t f = __builtin_amdgcn_bitop3_b32(x[c], y[c], r, 0xE8);
            y[c] = r + f + y[c];
            x[c] = f ^ (uint32_t)it;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c) acc ^= x[c] + y[c];
    sink[blockIdx.x * WGSIZE + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cycles[blockIdx.x * (WGSIZE / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int WGSIZE>
int run(int grid, std::string& out) {
    uint32_t* sink;
    uint64_t* cyc;
    const int waves = grid * WGSIZE / 64;
    CK(hipMalloc(&sink, (size_t)grid * WGSIZE * 4));
    CK(hipMalloc(&cyc, (size_t)waves * 8));
    for (int rep = 0; rep < 2; ++rep) {  // first launch warms up
        hipLaunchKernelGGL(valu_kernel<WGSIZE>, dim3(grid), dim3(WGSIZE), 0, 0, 12345u, sink, cyc);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
    }
    std::vector<uint64_t> h(waves);
    CK(hipMemcpy(h.data(), cyc, waves * 8, hipMemcpyDeviceToHost));
    std::sort(h.begin(), h.end());
    const double ops = (double)kIter * kChains * 4;
    char b[200];
    std::snprintf(b, sizeof b, "%s\"wg%d_grid%d\": {\"waves_per_simd\": %d, \"cycles_per_valu_median\": %.3f, "
                  "\"cycles_per_valu_min\": %.3f}",
                  out.size() > 1 ? ", " : "", WGSIZE, grid, WGSIZE / 256, h[waves / 2] / ops, h[0] / ops);
    out += b;
    CK(hipFree(sink));
    CK(hipFree(cyc));
    return 0;
}

int main() {
    std::string out = "{";
    // 8 workgroups: one per CU on 8 CUs (dispatch spreads them over XCDs/CUs)
    if (run<256>(8, out) || run<512>(8, out) || run<1024>(8, out)) return 1;
    // full chip, one wave per SIMD (power-capped regime) for comparison
    if (run<256>(256, out) || run<512>(256, out)) return 1;
    out += ", \"note\": \"s_memtime counts shader clock cycles; 32 VALU per iteration per chain-set\"}";
    std::printf("%s\n", out.c_str());
    return 0;
}
