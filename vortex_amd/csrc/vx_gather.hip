// vx_gather.hip — pull scattered pieces out of registered host memory into a
// slot's HBM arena with one kernel.
//
// vortex's completed pieces sit in unrelated BufferPool buffers
// (buf_pool.rs:92-133), so a batch is many small, non-adjacent host ranges.
// One hipMemcpyAsync per piece moves 256 KiB pieces at only 16.7 GiB/s (the
// per-call cost), while a kernel reading the pieces through the device
// mapping of the registered pool runs at the flat-DMA rate: 53.5 GiB/s for
// scattered 16 KiB, 256 KiB and 2 MiB pieces alike
// (a round-1 probe: profiles/r01/h2d/gather.json).
//
// Work is cut into 64 KiB tiles: piece i owns tiles [tfirst[i], tfirst[i+1])
// (a prefix built at submit; pieces not gathered own none).  A workgroup takes
// a tile, finds its piece by binary search on the prefix (wave-uniform), and
// copies it with 16-byte loads, four in flight per lane; the < 16-byte tail
// goes byte by byte.  Sources are 16-byte aligned (checked at submit).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vx_kernels.h"

namespace vx {

constexpr uint32_t kGatherTile = 64 * 1024;
constexpr int kGatherBlock = 256;
constexpr int kGatherGrid = 64;  // workgroups per launch (see the note above launch_gather)

__global__ __launch_bounds__(kGatherBlock) void gather_kernel(const uint64_t* __restrict__ src,
                                                              const uint64_t* __restrict__ dst_off,
                                                              const uint32_t* __restrict__ lens,
                                                              const uint32_t* __restrict__ tfirst, uint32_t n,
                                                              uint8_t* __restrict__ arena) {
    const uint32_t ntiles = tfirst[n];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        // last piece p with tfirst[p] <= t (pieces with no tiles are skipped)
        uint32_t lo = 0, hi = n;  // invariant: tfirst[lo] <= t < tfirst[hi]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) / 2;
            if (tfirst[mid] <= t) lo = mid;
            else hi = mid;
        }
        const uint32_t p = lo;
        const uint64_t off = (uint64_t)(t - tfirst[p]) * kGatherTile;
        const uint32_t len = (uint32_t)min<uint64_t>(kGatherTile, lens[p] - off);
        const uint8_t* s = reinterpret_cast<const uint8_t*>(src[p]) + off;
        uint8_t* d = arena + dst_off[p] + off;
        const uint32_t words = len / 16;
        const uint4* s4 = reinterpret_cast<const uint4*>(s);
        uint4* d4 = reinterpret_cast<uint4*>(d);
        constexpr int U = 4;
        for (uint32_t i = threadIdx.x; i < words; i += kGatherBlock * U) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t j = i + u * kGatherBlock;
                if (j < words) v[u] = s4[j];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t j = i + u * kGatherBlock;
                if (j < words) d4[j] = v[u];
            }
        }
        const uint32_t tail = len - words * 16;
        if (threadIdx.x < tail) d[words * 16 + threadIdx.x] = s[words * 16 + threadIdx.x];
    }
}

uint32_t gather_tiles(uint32_t len) { return (len + kGatherTile - 1) / kGatherTile; }

// Grid size.  64 workgroups already move 52.8 GiB/s alone (256: 52.8, 32:
// 52.3; profiles/r01/h2d/gather3.json), and a gather runs BESIDE hash kernels
// (the next chunk round, other slots).  With 256 workgroups the slow host
// reads in flight starved a concurrent chunk kernel's HBM loads: the kernel
// took 1.74 ms instead of 0.83 (rocprofv3 trace, profiles/r01/async/), and
// one-mmap-per-piece 2 MiB batches ran at 35 GiB/s.  At 64: 49.4 GiB/s; async
// 256 KiB pieces 42 -> 47 GiB/s.

hipError_t launch_gather(const uint64_t* src, const uint64_t* dst_off, const uint32_t* lens, const uint32_t* tfirst,
                         uint32_t n, uint32_t ntiles, uint8_t* arena, hipStream_t stream, uint32_t max_grid) {
    if (n == 0 || ntiles == 0) return hipSuccess;
    const uint32_t cap = max_grid ? max_grid : (uint32_t)kGatherGrid;
    const uint32_t grid = ntiles < cap ? ntiles : cap;
    hipLaunchKernelGGL(gather_kernel, dim3(grid), dim3(kGatherBlock), 0, stream, src, dst_off, lens, tfirst, n,
                       arena);
    return hipGetLastError();
}

}  // namespace vx
