// energy_probe.hip — is any SHA-1 op cheaper in energy than another?
//
// The config-2 kernel runs one wave per SIMD on all 1,024 SIMDs at the
// 1,400 W board cap, where the clock (2.0-2.25 GHz) and so the op rate are
// set by energy per op.  Each variant here runs one stream of
// independent VALU ops of a single kind, one wave on every SIMD, for ~2 s so
// the cap engages, and reports the whole-chip op rate (wall clock, HIP
// events) next to the cycles per op the waves saw (s_memtime).  Under the cap
// a cheaper op shows up as a higher clock and so a higher rate at the same
// cycles per op.
//   xor_bitop3   v_bitop3_b32 a, b, b (0x3c): what hipcc emits for the schedule's 2-input xor
//   xor_vop2     v_xor_b32_e32 (the 4-byte form)
//   xor3_bitop3  v_bitop3_b32 0x96 (3 sources)
//   add3         v_add3_u32
//   alignbit     v_alignbit_b32 (rotate)
//   perm         v_perm_b32 (byte swap)
//   sha_mix      the round's mix: add3 / alignbit / bitop3 / alignbit / add3
//   idle_nop     s_nop 0 only (issue slots with no VALU work)
//   *_2_waves_per_simd  the same stream with two waves on every SIMD
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define REP8(x) x x x x x x x x
#define BODY(b) REP8(b) REP8(b) REP8(b) b b b b b b  // 30 x 8 = 240 instructions

#define BXB "v_bitop3_b32 v64, v41, v42, v42 bitop3:0x3c\n v_bitop3_b32 v65, v43, v44, v44 bitop3:0x3c\n v_bitop3_b32 v66, v45, v46, v46 bitop3:0x3c\n v_bitop3_b32 v67, v47, v41, v41 bitop3:0x3c\n v_bitop3_b32 v68, v42, v43, v43 bitop3:0x3c\n v_bitop3_b32 v69, v44, v45, v45 bitop3:0x3c\n v_bitop3_b32 v70, v46, v47, v47 bitop3:0x3c\n v_bitop3_b32 v71, v41, v43, v43 bitop3:0x3c\n"
#define BXV "v_xor_b32_e32 v64, v41, v42\n v_xor_b32_e32 v65, v43, v44\n v_xor_b32_e32 v66, v45, v46\n v_xor_b32_e32 v67, v47, v41\n v_xor_b32_e32 v68, v42, v43\n v_xor_b32_e32 v69, v44, v45\n v_xor_b32_e32 v70, v46, v47\n v_xor_b32_e32 v71, v41, v43\n"
#define BX3 "v_bitop3_b32 v64, v41, v42, v43 bitop3:0x96\n v_bitop3_b32 v65, v44, v45, v46 bitop3:0x96\n v_bitop3_b32 v66, v47, v41, v42 bitop3:0x96\n v_bitop3_b32 v67, v43, v44, v45 bitop3:0x96\n v_bitop3_b32 v68, v46, v47, v41 bitop3:0x96\n v_bitop3_b32 v69, v42, v43, v44 bitop3:0x96\n v_bitop3_b32 v70, v45, v46, v47 bitop3:0x96\n v_bitop3_b32 v71, v41, v44, v47 bitop3:0x96\n"
#define BA3 "v_add3_u32 v64, v41, v42, v43\n v_add3_u32 v65, v44, v45, v46\n v_add3_u32 v66, v47, v41, v42\n v_add3_u32 v67, v43, v44, v45\n v_add3_u32 v68, v46, v47, v41\n v_add3_u32 v69, v42, v43, v44\n v_add3_u32 v70, v45, v46, v47\n v_add3_u32 v71, v41, v44, v47\n"
#define BAL "v_alignbit_b32 v64, v41, v41, 27\n v_add_u32_e32 v72, v42, v43\n v_alignbit_b32 v65, v44, v44, 2\n v_add_u32_e32 v73, v45, v46\n v_alignbit_b32 v66, v47, v47, 27\n v_add_u32_e32 v74, v41, v42\n v_alignbit_b32 v67, v43, v43, 2\n v_add_u32_e32 v75, v44, v45\n"
#define BAV "v_add_u32_e32 v72, v42, v43\n v_add_u32_e32 v73, v45, v46\n v_add_u32_e32 v74, v41, v42\n v_add_u32_e32 v75, v44, v45\n v_add_u32_e32 v72, v46, v43\n v_add_u32_e32 v73, v47, v46\n v_add_u32_e32 v74, v43, v42\n v_add_u32_e32 v75, v41, v45\n"
#define BPM "v_perm_b32 v64, v41, v41, s40\n v_perm_b32 v65, v42, v42, s40\n v_perm_b32 v66, v43, v43, s40\n v_perm_b32 v67, v44, v44, s40\n v_perm_b32 v68, v45, v45, s40\n v_perm_b32 v69, v46, v46, s40\n v_perm_b32 v70, v47, v47, s40\n v_perm_b32 v71, v41, v42, s40\n"
#define BMX "v_add3_u32 v64, v41, v42, v43\n v_alignbit_b32 v65, v44, v44, 27\n v_bitop3_b32 v66, v41, v42, v43 bitop3:0xca\n v_alignbit_b32 v67, v45, v45, 2\n v_add3_u32 v68, v45, v46, v47\n v_alignbit_b32 v69, v42, v42, 27\n v_bitop3_b32 v70, v45, v46, v47 bitop3:0x96\n v_add3_u32 v71, v41, v46, v43\n"
#define BNP "s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n"

#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "s40"

template <int T>
__global__ __launch_bounds__(512) void probe(uint32_t iters, unsigned long long* cyc, uint32_t seed) {
    // random-looking operands so the datapath toggles like real data
    const uint32_t x = (threadIdx.x + 1) * 0x9E3779B9u ^ seed * 0x85EBCA6Bu ^ blockIdx.x * 0xC2B2AE35u;
    asm volatile("v_mov_b32 v41, %0\n v_mul_lo_u32 v42, v41, v41\n s_mov_b32 s40, 0x55aa55aa\n v_xor_b32 v43, s40, v42\n"
                 "v_mul_lo_u32 v44, v43, v41\n v_add_u32 v45, v44, v42\n v_mul_lo_u32 v46, v45, v43\n"
                 "v_xor_b32 v47, v46, v41\n s_mov_b32 s40, 0x00010203" ::"v"(x) : CLOB);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < iters; ++i) {
        if (T == 0) asm volatile(".p2align 5\n" BODY(BXB) ::: CLOB);
        if (T == 1) asm volatile(".p2align 5\n" BODY(BXV) ::: CLOB);
        if (T == 2) asm volatile(".p2align 5\n" BODY(BX3) ::: CLOB);
        if (T == 3) asm volatile(".p2align 5\n" BODY(BA3) ::: CLOB);
        if (T == 4) asm volatile(".p2align 5\n" BODY(BAL) ::: CLOB);
        if (T == 5) asm volatile(".p2align 5\n" BODY(BAV) ::: CLOB);
        if (T == 6) asm volatile(".p2align 5\n" BODY(BPM) ::: CLOB);
        if (T == 7) asm volatile(".p2align 5\n" BODY(BMX) ::: CLOB);
        if (T == 8) asm volatile(".p2align 5\n" BODY(BNP) ::: CLOB);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
}

template <int T>
static void run(const char* name, unsigned long long* dc, double target_s, bool comma, int wps = 1) {
    const int G = 256;  // 256 workgroups x 4 waves = one wave on each of the 1,024 SIMDs (x wps waves per SIMD)
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    // calibrate: a short run, then size the long one to ~target_s
    uint32_t iters = 2000;
    float ms = 0;
    for (int pass = 0; pass < 2; ++pass) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL(probe<T>, dim3(G), dim3(256 * wps), 0, 0, iters, dc, 7u);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
        if (pass == 0) iters = (uint32_t)std::min(4.0e9, iters * (target_s * 1e3 / std::max(ms, 0.01f)));
    }
    std::vector<unsigned long long> all(G * 8), c;
    (void)hipMemcpy(all.data(), dc, G * 8 * 8, hipMemcpyDeviceToHost);
    for (int g = 0; g < G; ++g)
        for (int w = 0; w < 4 * wps; ++w) c.push_back(all[g * 8 + w]);
    std::sort(c.begin(), c.end());
    const double ops = (double)iters * 240.0;              // per wave
    const double cyc_per_op = (double)c[c.size() / 2] / ops;
    const double wave_ops_per_s = ops * G * 4 * wps / (ms * 1e-3);  // wave-instructions per second, whole chip
    const double clock_ghz = cyc_per_op * ops / (ms * 1e-3) / 1e9;
    std::printf("%s\"%s\": {\"s\": %.3f, \"cycles_per_op\": %.3f, \"clock_GHz\": %.3f, \"chip_Gwaveops_per_s\": %.2f}",
                comma ? ", " : "", name, ms * 1e-3, cyc_per_op, clock_ghz, wave_ops_per_s / 1e9);
    std::fflush(stdout);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
}

int main(int argc, char** argv) {
    const double t = argc > 1 ? std::atof(argv[1]) : 2.0;
    unsigned long long* dc = nullptr;
    if (hipMalloc(&dc, 256 * 8 * 8) != hipSuccess) return 1;
    std::printf("{\"unit\": \"one wave per SIMD on all SIMDs, ~%.1f s per variant\"", t);
    run<7>("sha_mix", dc, t, true);
    run<0>("xor_bitop3", dc, t, true);
    run<1>("xor_vop2", dc, t, true);
    run<2>("xor3_bitop3", dc, t, true);
    run<3>("add3", dc, t, true);
    run<4>("alignbit_add_vop2_alt", dc, t, true);
    run<5>("add_vop2", dc, t, true);
    run<6>("perm", dc, t, true);
    run<8>("idle_nop", dc, t, true);
    run<7>("sha_mix_again", dc, t, true);
    run<7>("sha_mix_2_waves_per_simd", dc, t, true, 2);
    run<1>("xor_vop2_2_waves_per_simd", dc, t, true, 2);
    run<5>("add_vop2_2_waves_per_simd", dc, t, true, 2);
    run<3>("add3_2_waves_per_simd", dc, t, true, 2);
    std::printf("}\n");
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
