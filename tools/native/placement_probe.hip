// placement_probe.hip — where does the dispatcher put the split kernel's
// workgroups (2 waves of 64, LDS 40 KiB or 60 KiB) when a launch has only a
// few of them?  Each wave records XCC_ID and HW_ID (CU, SIMD, wave slot) and
// spins ~200 µs so the whole grid is co-resident, like a chain-bound launch.
// Prints, per LDS size and grid: workgroups per CU (max / distinct CUs) and
// how many workgroups have both waves on ONE SIMD.  One JSON line.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));        \
            return 1;                                                           \
        }                                                                       \
    } while (0)

template <int LDS_BYTES>
__global__ __launch_bounds__(128) void where_kernel(uint32_t* out, uint32_t spin) {
    __shared__ uint32_t pad[LDS_BYTES / 4];
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    pad[threadIdx.x] = hw;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < spin) __builtin_amdgcn_s_sleep(2);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        const uint32_t w = blockIdx.x * 2 + threadIdx.x / 64;
        out[2 * w] = hw + pad[(threadIdx.x + 64) & 127] * 0;  // keep the LDS allocation
        out[2 * w + 1] = xcc;
    }
}

template <int LDS_BYTES>
int run(int grid, std::string& js) {
    uint32_t* d;
    CK(hipMalloc(&d, grid * 2 * 2 * 4));
    hipLaunchKernelGGL(where_kernel<LDS_BYTES>, dim3(grid), dim3(128), 0, 0, d, 200000u);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> h(grid * 4);
    CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
    CK(hipFree(d));
    // gfx9 HW_ID: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13]
    std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, int> per_cu;
    int same_simd = 0;
    for (int b = 0; b < grid; ++b) {
        uint32_t hw0 = h[4 * b], x0 = h[4 * b + 1], hw1 = h[4 * b + 2];
        auto cu = std::make_tuple(x0 & 0xF, (hw0 >> 13) & 7, (hw0 >> 12) & 1, (hw0 >> 8) & 0xF);
        per_cu[cu]++;
        if (((hw0 >> 4) & 3) == ((hw1 >> 4) & 3)) ++same_simd;
    }
    int mx = 0;
    for (auto& kv : per_cu) mx = std::max(mx, kv.second);
    char buf[256];
    std::snprintf(buf, sizeof buf, "%s\"lds%dK_grid%d\": {\"cus_used\": %zu, \"max_wg_per_cu\": %d, "
                  "\"wg_with_both_waves_on_one_simd\": %d}",
                  js.size() > 1 ? ", " : "", LDS_BYTES / 1024, grid, per_cu.size(), mx, same_simd);
    js += buf;
    return 0;
}

int main() {
    std::string js = "{";
    for (int grid : {22, 128, 256, 512}) {
        if (run<40 * 1024>(grid, js) || run<60 * 1024>(grid, js)) return 1;
    }
    js += "}";
    std::printf("%s\n", js.c_str());
    return 0;
}
