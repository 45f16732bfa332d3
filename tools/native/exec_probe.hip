// exec_probe.hip — does a lone wave's VALU issue cost on gfx950 depend on how
// many lanes are live?  A CDNA4 SIMD is 32 lanes wide and a wave64 VALU op
// takes two passes, but one wave alone sustains ~4 cycles per op
// (valu_issue_probe).  If a wave whose EXEC covers only one 32-lane half
// issued faster, a chain-bound launch (few long pieces, one lane per piece)
// could run its lanes in half-waves.
//
// Each body is 240 independent or dependent ops (fixed registers, inline asm);
// the asm sets EXEC to the requested mask on entry and restores it on exit, so
// the compiler's own code runs with the full mask.  One wave per workgroup,
// 64 workgroups, s_memtime around the loop, median over waves; prints cycles
// per instruction.  `waves` > 1 puts that many waves in one workgroup (same
// CU, one per SIMD up to 4, then two per SIMD).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define REP8(x) x x x x x x x x
#define BODY(b) REP8(b) REP8(b) REP8(b) b b b b b b  // 30 x 8 = 240 instructions

// independent SHA-1-like mix (same as valu_issue_probe's sha_mix)
#define BM "v_add3_u32 v64, v41, v42, v43\n v_alignbit_b32 v65, v44, v44, 27\n v_bitop3_b32 v66, v41, v42, v43 bitop3:0xca\n v_alignbit_b32 v67, v45, v45, 2\n v_add3_u32 v68, v45, v46, v47\n v_alignbit_b32 v69, v42, v42, 27\n v_bitop3_b32 v70, v45, v46, v47 bitop3:0x96\n v_add3_u32 v71, v41, v46, v43\n"
// dependent add3 chain
#define BD "v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n v_add3_u32 v64, v64, v41, v42\n"
// independent v_add_u32_e32 (VOP2)
#define BV "v_add_u32_e32 v64, v41, v42\n v_add_u32_e32 v65, v41, v42\n v_add_u32_e32 v66, v41, v42\n v_add_u32_e32 v67, v41, v42\n v_add_u32_e32 v68, v41, v42\n v_add_u32_e32 v69, v41, v42\n v_add_u32_e32 v70, v41, v42\n v_add_u32_e32 v71, v41, v42\n"

#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "s40", "s41"

template <int T>
__global__ __launch_bounds__(512) void probe(uint32_t iters, uint64_t mask, unsigned long long* cyc) {
    asm volatile("v_mov_b32 v40, 1\n v_mov_b32 v41, 2\n v_mov_b32 v42, 3\n v_mov_b32 v43, 4\n v_mov_b32 v44, 5\n"
                 "v_mov_b32 v45, 6\n v_mov_b32 v46, 7\n v_mov_b32 v47, 8\n v_mov_b32 v48, 9\n v_mov_b32 v64, 0\n"
                 "v_mov_b32 v65, 0" ::: CLOB);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < iters; ++i) {
#define RUN(b) asm volatile("s_mov_b64 s[40:41], exec\n s_mov_b64 exec, %0\n" BODY(b) "s_mov_b64 exec, s[40:41]\n" ::"s"(mask) : CLOB)
        if (T == 0) RUN(BM);
        if (T == 1) RUN(BD);
        if (T == 2) RUN(BV);
#undef RUN
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
}

template <int T>
static void run(const char* name, unsigned long long* dc, int waves, uint64_t mask, bool comma) {
    const int G = 64;
    const uint32_t iters = 20000;
    hipLaunchKernelGGL(probe<T>, dim3(G), dim3(64 * waves), 0, 0, 200u, mask, dc);
    hipLaunchKernelGGL(probe<T>, dim3(G), dim3(64 * waves), 0, 0, iters, mask, dc);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> c(G * 8), v;
    (void)hipMemcpy(c.data(), dc, G * 8 * 8, hipMemcpyDeviceToHost);
    for (int g = 0; g < G; ++g)
        for (int w = 0; w < waves; ++w) v.push_back(c[g * 8 + w]);
    std::sort(v.begin(), v.end());
    std::printf("%s\"%s_w%d_m%016llx\": %.3f", comma ? ", " : "", name, waves, (unsigned long long)mask,
                (double)v[v.size() / 2] / (iters * 240.0));
    std::fflush(stdout);
}

int main() {
    unsigned long long* dc = nullptr;
    if (hipMalloc(&dc, 64 * 8 * 8) != hipSuccess) return 1;
    const uint64_t masks[] = {~0ull, 0xffffffffull, 0xffffffff00000000ull, 0xffffull, 1ull};
    std::printf("{\"unit\": \"cycles per instruction per wave\"");
    for (int waves : {1, 4, 8})
        for (uint64_t m : masks) {
            run<0>("sha_mix", dc, waves, m, true);
            run<1>("add3_dep", dc, waves, m, true);
            run<2>("add_vop2", dc, waves, m, true);
        }
    std::printf("}\n");
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
