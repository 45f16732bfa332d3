// gather_probe.hip — can a kernel pull scattered pieces out of registered
// host memory as fast as the DMA engines move one flat buffer?
//
// The async download path hands over pieces that sit in scattered pool
// buffers (buf_pool.rs), so each one is its own hipMemcpyAsync today
// (9.8-16.5 GiB/s at 128-256 KiB per copy, profiles/r01/h2d/h2d2d.json).  This
// measures a gather kernel that reads the pieces through the mapped device
// pointer of a hipHostRegister'd mmap (zero-copy over PCIe) and writes them
// densely into HBM, for several piece sizes and grid sizes, against one flat
// hipMemcpyAsync of the same bytes.  Prints one JSON line (GiB/s, best of 3).
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <random>
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

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One workgroup copies `per_wg` bytes of one piece per step; piece p's bytes
// come from src + src_off[p] and land at dst + p * len.  dwordx4 per lane,
// U loads in flight per lane before the stores.
template <int U>
__global__ __launch_bounds__(256) void gather_kernel(const uint8_t* __restrict__ src,
                                                     const uint64_t* __restrict__ src_off, uint8_t* __restrict__ dst,
                                                     uint64_t len, uint64_t n, uint64_t tile) {
    const uint64_t tiles_per_piece = len / tile;
    const uint64_t ntiles = n * tiles_per_piece;
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t p = t / tiles_per_piece, k = t % tiles_per_piece;
        const uint4* s = reinterpret_cast<const uint4*>(src + src_off[p] + k * tile);
        uint4* d = reinterpret_cast<uint4*>(dst + p * len + k * tile);
        const uint64_t words = tile / 16;
        for (uint64_t i = threadIdx.x; i < words; i += 256 * U) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t j = i + (uint64_t)u * 256;
                if (j < words) v[u] = s[j];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t j = i + (uint64_t)u * 256;
                if (j < words) d[j] = v[u];
            }
        }
    }
}

int main() {
    const size_t bytes = 2ull << 30;
    uint8_t* d = nullptr;
    CK(hipMalloc(&d, bytes));
    // host pool: 2x the bytes so the scattered pieces are spread out
    const size_t pool = 2 * bytes;
    uint8_t* mm = static_cast<uint8_t*>(mmap(nullptr, pool, PROT_READ | PROT_WRITE,
                                              MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0));
    std::memset(mm, 1, pool);
    CK(hipHostRegister(mm, pool, hipHostRegisterMapped));
    uint8_t* dmm = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dmm), mm, 0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint64_t* d_off = nullptr;
    CK(hipMalloc(&d_off, (bytes / 16384) * 8));
    std::string out = "{";
    auto emit = [&](const std::string& k, double v) {
        char b[128];
        std::snprintf(b, sizeof b, "%s\"%s\": %.2f", out.size() > 1 ? ", " : "", k.c_str(), v);
        out += b;
    };
    CK(hipMemcpyAsync(d, mm, 64 << 20, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    {
        double best = 0;
        for (int rep = 0; rep < 3; ++rep) {
            const double t0 = now();
            CK(hipMemcpyAsync(d, mm, bytes, hipMemcpyHostToDevice, st));
            CK(hipStreamSynchronize(st));
            best = std::max(best, bytes / (now() - t0) / (1 << 30));
        }
        emit("flat_dma", best);
    }
    std::mt19937_64 rng(7);
    for (size_t L : {size_t(16) << 10, size_t(256) << 10, size_t(2) << 20}) {
        const size_t n = bytes / L, slots = pool / L;
        std::vector<uint64_t> slot(slots);
        std::iota(slot.begin(), slot.end(), 0);
        std::shuffle(slot.begin(), slot.end(), rng);
        std::vector<uint64_t> off(n);
        for (size_t i = 0; i < n; ++i) off[i] = slot[i] * L;
        CK(hipMemcpy(d_off, off.data(), n * 8, hipMemcpyHostToDevice));
        const std::string tag = std::to_string(L >> 10) + "K";
        for (int grid : {32, 64, 256, 1024}) {
            for (uint64_t tile : {uint64_t(16) << 10}) {
                double best = 0;
                for (int rep = 0; rep < 3; ++rep) {
                    const double t0 = now();
                    hipLaunchKernelGGL((gather_kernel<4>), dim3(grid), dim3(256), 0, st, dmm, d_off, d, L, n, tile);
                    CK(hipGetLastError());
                    CK(hipStreamSynchronize(st));
                    best = std::max(best, bytes / (now() - t0) / (1 << 30));
                }
                emit("kernel_" + tag + "_g" + std::to_string(grid), best);
            }
        }
        // one hipMemcpyBatchAsync of the same scattered pieces (SDMA, no CUs)
        {
            std::vector<void*> dsts(n), srcs(n);
            std::vector<size_t> sizes(n, L);
            for (size_t i = 0; i < n; ++i) {
                dsts[i] = d + i * L;
                srcs[i] = mm + off[i];
            }
            double best = 0;
            for (int rep = 0; rep < 3; ++rep) {
                size_t fail_idx = 0;
                const double t0 = now();
                CK(hipMemcpyBatchAsync(dsts.data(), srcs.data(), sizes.data(), n, nullptr, nullptr, 0, &fail_idx, st));
                CK(hipStreamSynchronize(st));
                best = std::max(best, bytes / (now() - t0) / (1 << 30));
            }
            emit("batchdma_" + tag, best);
        }
        // per-piece DMA of the same scattered pieces (bounded call count)
        if (n <= 8192) {
            double best = 0;
            for (int rep = 0; rep < 3; ++rep) {
                const double t0 = now();
                for (size_t i = 0; i < n; ++i)
                    CK(hipMemcpyAsync(d + i * L, mm + off[i], L, hipMemcpyHostToDevice, st));
                CK(hipStreamSynchronize(st));
                best = std::max(best, bytes / (now() - t0) / (1 << 30));
            }
            emit("perpiece_dma_" + tag, best);
        }
        // check the gather moved the right bytes (first and last piece)
        std::vector<uint8_t> h(L);
        std::memset(mm + off[n - 1], 0x5A, 64);
        hipLaunchKernelGGL((gather_kernel<4>), dim3(1024), dim3(256), 0, st, dmm, d_off, d, L, n, uint64_t(16) << 10);
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(h.data(), d + (n - 1) * L, L, hipMemcpyDeviceToHost));
        if (h[0] != 0x5A || h[63] != 0x5A || h[64] != 1) {
            std::fprintf(stderr, "gather check failed at %s\n", tag.c_str());
            return 2;
        }
        std::memset(mm + off[n - 1], 1, 64);
    }
    out += "}";
    std::printf("%s\n", out.c_str());
    CK(hipHostUnregister(mm));
    munmap(mm, pool);
    CK(hipFree(d_off));
    CK(hipFree(d));
    return 0;
}
