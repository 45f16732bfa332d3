// valu_issue_probe.hip — what a lone wave's VALU stream costs per
// instruction on gfx950, by operand banks, encoding size and dependence.
//
// The split kernel's rounds-only consumer wave runs at ~4.5 cycles per VALU
// whatever the order of a round's ops (tools/native/rounds_sched_probe.hip),
// above the 4-cycle issue of one wave (MI355X_MICROARCH.md).  Each test is one
// inline-asm body of 240 instructions with fixed registers (asm bodies are long
// so the compiler's per-asm hazard padding is negligible), looped, one wave
// per workgroup on 64 workgroups; s_memtime around the loop; prints cycles
// per instruction (median over waves).
//   add3_banks3     v_add3_u32 with its 3 sources in 3 different VGPR banks (reg % 4)
//   add3_bank_same  v_add3_u32 with all 3 sources in one bank
//   add3_dep        each v_add3_u32 reads the previous result (dependent chain)
//   add3_dep2       dependence distance 2 (two interleaved chains)
//   alignbit_same   v_alignbit_b32 vD, vS, vS, 27 (a rotate: one register twice)
//   bitop3_banks3   v_bitop3_b32, sources in 3 banks
//   add_vop2        v_add_u32_e32 (4-byte encoding), independent
//   sha_mix         add3 / alignbit / bitop3 / alignbit / add3, independent
//   alignbit_two_regs                 v_alignbit_b32 with two different sources
//   add3_then_alignbit_of_it          alignbit reads the add3 issued right before it
//   alignbit_then_add3_of_it          add3 reads the alignbit issued right before it
//   alignbit_dep_chain                each alignbit rotates the previous result
//   alignbit_add3_alternating_indep   alternating, independent
//   bitop3_dep_chain                  each bitop3 reads the previous result
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#define REP8(x) x x x x x x x x

// 16 rotating destinations v64..v79 would need a generator; instead each test
// body repeats a block of 8 instructions whose destinations are v64..v71 and
// whose sources are v40..v47 (never written), so nothing depends on anything
// unless the test says so.
#define B3 "v_add3_u32 v64, v41, v42, v43\n v_add3_u32 v65, v41, v42, v43\n v_add3_u32 v66, v41, v42, v43\n v_add3_u32 v67, v41, v42, v43\n v_add3_u32 v68, v41, v42, v43\n v_add3_u32 v69, v41, v42, v43\n v_add3_u32 v70, v41, v42, v43\n v_add3_u32 v71, v41, v42, v43\n"
#define BS "v_add3_u32 v64, v40, v44, v48\n v_add3_u32 v65, v40, v44, v48\n v_add3_u32 v66, v40, v44, v48\n v_add3_u32 v67, v40, v44, v48\n v_add3_u32 v68, v40, v44, v48\n v_add3_u32 v69, v40, v44, v48\n v_add3_u32 v70, v40, v44, v48\n v_add3_u32 v71, v40, v44, v48\n"
#define BD "v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n"
#define BD2 "v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v65, v65, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v65, v65, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v65, v65, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v65, v65, v41, v42\n"
#define BA "v_alignbit_b32 v64, v41, v41, 27\n v_alignbit_b32 v65, v42, v42, 27\n v_alignbit_b32 v66, v43, v43, 27\n v_alignbit_b32 v67, v44, v44, 27\n v_alignbit_b32 v68, v41, v41, 2\n v_alignbit_b32 v69, v42, v42, 2\n v_alignbit_b32 v70, v43, v43, 2\n v_alignbit_b32 v71, v44, v44, 2\n"
#define BB "v_bitop3_b32 v64, v41, v42, v43 bitop3:0xca\n v_bitop3_b32 v65, v41, v42, v43 bitop3:0xca\n v_bitop3_b32 v66, v41, v42, v43 bitop3:0x96\n v_bitop3_b32 v67, v41, v42, v43 bitop3:0x96\n v_bitop3_b32 v68, v41, v42, v43 bitop3:0xe8\n v_bitop3_b32 v69, v41, v42, v43 bitop3:0xe8\n v_bitop3_b32 v70, v41, v42, v43 bitop3:0xca\n v_bitop3_b32 v71, v41, v42, v43 bitop3:0xca\n"
#define BV "v_add_u32_e32 v64, v41, v42\n v_add_u32_e32 v65, v41, v42\n v_add_u32_e32 v66, v41, v42\n v_add_u32_e32 v67, v41, v42\n v_add_u32_e32 v68, v41, v42\n v_add_u32_e32 v69, v41, v42\n v_add_u32_e32 v70, v41, v42\n v_add_u32_e32 v71, v41, v42\n"
#define BM "v_add3_u32 v64, v41, v42, v43\n v_alignbit_b32 v65, v44, v44, 27\n v_bitop3_b32 v66, v41, v42, v43 bitop3:0xca\n v_alignbit_b32 v67, v45, v45, 2\n v_add3_u32 v68, v45, v46, v47\n v_alignbit_b32 v69, v42, v42, 27\n v_bitop3_b32 v70, v45, v46, v47 bitop3:0x96\n v_add3_u32 v71, v41, v46, v43\n"

#define BA2 "v_alignbit_b32 v64, v41, v42, 27\n v_alignbit_b32 v65, v42, v43, 27\n v_alignbit_b32 v66, v43, v44, 27\n v_alignbit_b32 v67, v44, v45, 27\n v_alignbit_b32 v68, v41, v42, 2\n v_alignbit_b32 v69, v42, v43, 2\n v_alignbit_b32 v70, v43, v44, 2\n v_alignbit_b32 v71, v44, v45, 2\n"
#define BAD "v_add3_u32 v64, v41, v42, v43\n v_alignbit_b32 v65, v64, v64, 27\n v_add3_u32 v66, v41, v42, v43\n v_alignbit_b32 v67, v66, v66, 27\n v_add3_u32 v68, v41, v42, v43\n v_alignbit_b32 v69, v68, v68, 27\n v_add3_u32 v70, v41, v42, v43\n v_alignbit_b32 v71, v70, v70, 27\n"
#define BDA "v_alignbit_b32 v64, v41, v41, 27\n v_add3_u32 v65, v64, v42, v43\n v_alignbit_b32 v66, v42, v42, 27\n v_add3_u32 v67, v66, v42, v43\n v_alignbit_b32 v68, v43, v43, 27\n v_add3_u32 v69, v68, v42, v43\n v_alignbit_b32 v70, v44, v44, 27\n v_add3_u32 v71, v70, v42, v43\n"
#define BAC "v_alignbit_b32 v64, v64, v64, 27\n v_alignbit_b32 v64, v64, v64, 27\n v_alignbit_b32 v64, v64, v64, 27\n v_alignbit_b32 v64, v64, v64, 27\n v_alignbit_b32 v64, v64, v64, 27\n v_alignbit_b32 v64, v64, v64, 27\n v_alignbit_b32 v64, v64, v64, 27\n v_alignbit_b32 v64, v64, v64, 27\n"
#define BAX "v_alignbit_b32 v64, v41, v41, 27\n v_add3_u32 v65, v41, v42, v43\n v_alignbit_b32 v66, v42, v42, 27\n v_add3_u32 v67, v41, v42, v43\n v_alignbit_b32 v68, v43, v43, 27\n v_add3_u32 v69, v41, v42, v43\n v_alignbit_b32 v70, v44, v44, 27\n v_add3_u32 v71, v41, v42, v43\n"
#define BBD "v_bitop3_b32 v64, v64, v42, v43 bitop3:0xca\n v_bitop3_b32 v64, v64, v42, v43 bitop3:0x96\n v_bitop3_b32 v64, v64, v42, v43 bitop3:0xe8\n v_bitop3_b32 v64, v64, v42, v43 bitop3:0xca\n v_bitop3_b32 v64, v64, v42, v43 bitop3:0xca\n v_bitop3_b32 v64, v64, v42, v43 bitop3:0x96\n v_bitop3_b32 v64, v64, v42, v43 bitop3:0xe8\n v_bitop3_b32 v64, v64, v42, v43 bitop3:0xca\n"

#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71"
#define BODY(b) REP8(b) REP8(b) REP8(b) b b b b b b  // 30 x 8 = 240 instructions

template <int T>
__global__ __launch_bounds__(64) void probe(uint32_t iters, unsigned long long* cyc) {
    asm volatile("v_mov_b32 v40, 1\n v_mov_b32 v41, 2\n v_mov_b32 v42, 3\n v_mov_b32 v43, 4\n v_mov_b32 v44, 5\n"
                 "v_mov_b32 v45, 6\n v_mov_b32 v46, 7\n v_mov_b32 v47, 8\n v_mov_b32 v48, 9\n v_mov_b32 v64, 0\n"
                 "v_mov_b32 v65, 0" ::: CLOB);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < iters; ++i) {
        if (T == 0) asm volatile(BODY(B3) ::: CLOB);
        if (T == 1) asm volatile(BODY(BS) ::: CLOB);
        if (T == 2) asm volatile(BODY(BD) ::: CLOB);
        if (T == 3) asm volatile(BODY(BD2) ::: CLOB);
        if (T == 4) asm volatile(BODY(BA) ::: CLOB);
        if (T == 5) asm volatile(BODY(BB) ::: CLOB);
        if (T == 6) asm volatile(BODY(BV) ::: CLOB);
        if (T == 7) asm volatile(BODY(BM) ::: CLOB);
        if (T == 8) asm volatile(BODY(BA2) ::: CLOB);
        if (T == 9) asm volatile(BODY(BAD) ::: CLOB);
        if (T == 10) asm volatile(BODY(BDA) ::: CLOB);
        if (T == 11) asm volatile(BODY(BAC) ::: CLOB);
        if (T == 12) asm volatile(BODY(BAX) ::: CLOB);
        if (T == 13) asm volatile(BODY(BBD) ::: CLOB);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int T>
static void run(const char* name, unsigned long long* dc, bool comma) {
    const int G = 64;
    const uint32_t iters = 20000;
    hipLaunchKernelGGL(probe<T>, dim3(G), dim3(64), 0, 0, 200u, dc);
    hipLaunchKernelGGL(probe<T>, dim3(G), dim3(64), 0, 0, iters, dc);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> c(G);
    (void)hipMemcpy(c.data(), dc, G * 8, hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    std::printf("%s\"%s\": %.3f", comma ? ", " : "", name, (double)c[G / 2] / (iters * 240.0));
}

int main() {
    unsigned long long* dc = nullptr;
    if (hipMalloc(&dc, 64 * 8) != hipSuccess) return 1;
    std::printf("{\"unit\": \"cycles per instruction, one wave per SIMD\", ");
    run<0>("add3_banks3", dc, false);
    run<1>("add3_bank_same", dc, true);
    run<2>("add3_dep", dc, true);
    run<3>("add3_dep2", dc, true);
    run<4>("alignbit_same", dc, true);
    run<5>("bitop3_banks3", dc, true);
    run<6>("add_vop2", dc, true);
    run<7>("sha_mix", dc, true);
    run<8>("alignbit_two_regs", dc, true);
    run<9>("add3_then_alignbit_of_it", dc, true);
    run<10>("alignbit_then_add3_of_it", dc, true);
    run<11>("alignbit_dep_chain", dc, true);
    run<12>("alignbit_add3_alternating_indep", dc, true);
    run<13>("bitop3_dep_chain", dc, true);
    std::printf("}\n");
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
