// zc_pattern_probe.hip — which per-instruction access pattern lets a kernel
// read registered host memory (zero-copy, over PCIe) at the DMA rate?
//
// Context: the hash kernels pointed at pinned host
// memory pull only ~36 GiB/s over PCIe with each lane loading its own piece
// 16 bytes at a time, against ~53 GiB/s for the gather kernel, whose wave
// instructions each read 1 KiB contiguous.  A zero-copy producer could load
// cooperatively instead: G lanes per piece, 64/G pieces per instruction,
// G*16 contiguous bytes of each.  This probe streams 64 pieces per wave with
// each G (1 = the hash kernels' pattern, 64 = the gather's), 32 loads in
// flight per lane (kBatch), at several wave counts, and prints one JSON line per
// point (GiB/s, best of 3) next to a flat pinned copy of the same bytes.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));   \
            return 1;                                                      \
        }                                                                  \
    } while (0)

constexpr uint32_t kStep = 1024;                  // bytes of each piece per step
constexpr uint32_t kInstr = 64 * kStep / 1024;      // 64 wave-instructions (1 KiB each) per step
constexpr uint32_t kBatch = 32;                     // of which this many are in flight at once

// One wave (blockDim 64) streams pieces [64*blockIdx.x, +64) of length L.
// Instruction i of a step covers P = 64/G pieces, G*16 bytes of each.
template <int G>
__global__ __launch_bounds__(64) void zc_read(const uint8_t* __restrict__ pool, const uint64_t* __restrict__ off,
                                              uint64_t L, uint32_t* __restrict__ out) {
    constexpr int P = 64 / G;
    constexpr uint32_t per_group = kStep / (G * 16);  // instructions per piece group per step
    const int lane = threadIdx.x;
    const uint64_t p0 = (uint64_t)blockIdx.x * 64;
    uint32_t acc = 0;
    for (uint64_t s = 0; s < L; s += kStep) {
#pragma unroll
        for (uint32_t h = 0; h < kInstr; h += kBatch) {
            uint4 v[kBatch];
#pragma unroll
            for (uint32_t k = 0; k < kBatch; ++k) {
                const uint32_t i = h + k;
                const uint32_t pb = i / per_group;
                const uint32_t piece = pb * P + lane / G;
                const uint64_t o = s + (uint64_t)(i % per_group) * (G * 16) + (uint64_t)(lane % G) * 16;
                v[k] = *reinterpret_cast<const uint4*>(pool + off[p0 + piece] + o);
            }
#pragma unroll
            for (uint32_t k = 0; k < kBatch; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        }
    }
    out[blockIdx.x * 64 + lane] = acc;
}

template <int G>
hipError_t launch(const uint8_t* pool, const uint64_t* off, uint64_t L, uint32_t waves, uint32_t* out,
                  hipStream_t st) {
    hipLaunchKernelGGL(zc_read<G>, dim3(waves), dim3(64), 0, st, pool, off, L, out);
    return hipGetLastError();
}

int main(int argc, char** argv) {
    const uint64_t L = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 256 * 1024;
    const size_t pool_bytes = 4ull << 30;
    const uint64_t max_pieces = (pool_bytes / 2) / L;  // scattered over twice their bytes
    uint8_t* mm = static_cast<uint8_t*>(
        mmap(nullptr, pool_bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0));
    if (mm == MAP_FAILED) return 1;
    std::memset(mm, 7, pool_bytes);
    CK(hipHostRegister(mm, pool_bytes, hipHostRegisterMapped));
    uint8_t* dpool = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dpool), mm, 0));
    // piece slots of L bytes at random distinct positions in the pool
    std::vector<uint64_t> slots(pool_bytes / L);
    std::iota(slots.begin(), slots.end(), 0);
    std::mt19937_64 rng(42);
    std::shuffle(slots.begin(), slots.end(), rng);
    std::vector<uint64_t> off(max_pieces);
    for (uint64_t i = 0; i < max_pieces; ++i) off[i] = slots[i] * L;
    uint64_t* d_off = nullptr;
    uint32_t* d_out = nullptr;
    uint8_t* d_dst = nullptr;
    CK(hipMalloc(&d_off, max_pieces * 8));
    CK(hipMemcpy(d_off, off.data(), max_pieces * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_out, max_pieces * 4));
    CK(hipMalloc(&d_dst, 1ull << 30));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    auto timed = [&](auto&& fn, double& best) -> int {
        best = 1e30;
        for (int r = 0; r < 4; ++r) {
            CK(hipEventRecord(e0, st));
            CK(fn());
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0) best = std::min(best, (double)ms);  // first run warms up
        }
        return 0;
    };
    const double GiB = 1073741824.0;
    {
        double ms;
        if (timed([&] { return hipMemcpyAsync(d_dst, mm, 1ull << 30, hipMemcpyHostToDevice, st); }, ms)) return 1;
        std::printf("{\"case\": \"pinned_copy\", \"bytes\": %llu, \"ms\": %.3f, \"GiBps\": %.2f}\n", 1ull << 30, ms,
                    (1ull << 30) / (ms * 1e-3) / GiB);
    }
    const uint32_t wave_counts[] = {8, 32, 64, 128, 256, 512};
    for (uint32_t waves : wave_counts) {
        if ((uint64_t)waves * 64 > max_pieces) continue;
        const double bytes = (double)waves * 64 * L;
        for (int g : {1, 4, 16, 32, 64}) {
            double ms;
            auto fn = [&]() -> hipError_t {
                switch (g) {
                    case 1: return launch<1>(dpool, d_off, L, waves, d_out, st);
                    case 4: return launch<4>(dpool, d_off, L, waves, d_out, st);
                    case 16: return launch<16>(dpool, d_off, L, waves, d_out, st);
                    case 32: return launch<32>(dpool, d_off, L, waves, d_out, st);
                    default: return launch<64>(dpool, d_off, L, waves, d_out, st);
                }
            };
            if (timed(fn, ms)) return 1;
            std::printf("{\"case\": \"zc_read\", \"lanes_per_piece\": %d, \"waves\": %u, \"piece_len\": %llu, "
                        "\"ms\": %.3f, \"GiBps\": %.2f}\n",
                        g, waves, (unsigned long long)L, ms, bytes / (ms * 1e-3) / GiB);
            std::fflush(stdout);
        }
    }
    CK(hipHostUnregister(mm));
    munmap(mm, pool_bytes);
    return 0;
}
