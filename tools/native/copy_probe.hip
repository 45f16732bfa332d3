// copy_probe.hip — the warm re-verify's page cache -> pinned stage copy,
// three ways, with the H2D copy chain running beside it (diagnostic, not the
// product; EXPERIMENTS.md §6.1).  With the DMA running, the engine's readers
// copy out of the page cache at 2.6-4.7 GiB/s per thread against 6+ without
// it: host memory is shared by the page cache read, the stage write (plus its
// read for ownership) and the DMA read.  Question: does a user-space copy
// with non-temporal stores (no read for ownership, no cache pollution) move
// more bytes per second than the kernel's copy_to_user under the same DMA?
//   mode 0  pread into the stage (what vx_files::Readers does)
//   mode 1  mmap of the file, memcpy into the stage
//   mode 2  mmap of the file, 32-byte loads + streaming stores into the stage
// Rounds follow vx_verify_files: round r = bytes [r*C, (r+1)*C) of every
// piece, lanes 4 KiB-aligned in the stage; `threads` threads split a round's
// pieces; each finished round goes to the GPU with one hipMemcpyAsync while
// the next round is copied (stages round-robin, a stage reused only after its
// H2D completed).  mmap/munmap are inside the timed region.
//
// usage: copy_probe <file> <piece_len> <mode> [threads=16] [chunk=262144] [dma=1] [reps=3] [populate=0]
// Prints one JSON line: median GiB/s over reps and the DMA's busy fraction.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace {

__attribute__((target("avx2"))) void copy_nt(uint8_t* d, const uint8_t* s, size_t n) {
    size_t i = 0;
    if (((reinterpret_cast<uintptr_t>(d) | reinterpret_cast<uintptr_t>(s)) & 31) == 0) {
        for (; i + 128 <= n; i += 128) {
            const __m256i a = _mm256_load_si256(reinterpret_cast<const __m256i*>(s + i));
            const __m256i b = _mm256_load_si256(reinterpret_cast<const __m256i*>(s + i + 32));
            const __m256i c = _mm256_load_si256(reinterpret_cast<const __m256i*>(s + i + 64));
            const __m256i e = _mm256_load_si256(reinterpret_cast<const __m256i*>(s + i + 96));
            _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a);
            _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), b);
            _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), c);
            _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), e);
        }
    }
    std::memcpy(d + i, s + i, n - i);
}

bool pread_full(int fd, uint8_t* dst, int64_t off, int64_t len) {
    int64_t got = 0;
    while (got < len) {
        const ssize_t r = pread(fd, dst + got, (size_t)(len - got), off + got);
        if (r <= 0) return false;
        got += r;
    }
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const char* path = argv[1];
    const uint64_t pl = std::strtoull(argv[2], nullptr, 0);
    const int mode = std::atoi(argv[3]);
    const int threads = argc > 4 ? std::atoi(argv[4]) : 16;
    const uint64_t C = argc > 5 ? std::strtoull(argv[5], nullptr, 0) : 262144;
    const bool dma = argc > 6 ? std::atoi(argv[6]) != 0 : true;
    const int reps = argc > 7 ? std::atoi(argv[7]) : 3;
    const bool populate = argc > 8 && std::atoi(argv[8]) != 0;
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    struct stat st;
    if (fd < 0 || fstat(fd, &st) != 0 || pl == 0 || C == 0 || threads < 1 || mode < 0 || mode > 2) return 3;
    const uint64_t total = (uint64_t)st.st_size;
    const uint64_t n = (total + pl - 1) / pl;
    const uint64_t pitch = (C + 4095) / 4096 * 4096;
    const uint64_t stage_bytes = n * pitch;
    constexpr int kStages = 3;
    uint8_t* stage[kStages] = {};
    for (auto& s : stage)
        if (hipHostMalloc(&s, stage_bytes, hipHostMallocDefault) != hipSuccess) return 4;
    uint8_t* dev = nullptr;
    hipStream_t ds = nullptr;
    hipEvent_t done[kStages] = {}, beg[kStages] = {};
    if (dma) {
        if (hipMalloc(&dev, stage_bytes) != hipSuccess || hipStreamCreate(&ds) != hipSuccess) return 5;
        for (int k = 0; k < kStages; ++k)
            if (hipEventCreate(&done[k]) != hipSuccess || hipEventCreate(&beg[k]) != hipSuccess) return 5;
    }
    const uint64_t rounds = (pl + C - 1) / C;
    std::vector<double> rates, busy;
    for (int rep = 0; rep < reps; ++rep) {
        const auto t0 = std::chrono::steady_clock::now();
        const uint8_t* map = nullptr;
        if (mode > 0) {
            void* m = mmap(nullptr, total, PROT_READ, MAP_SHARED | (populate ? MAP_POPULATE : 0), fd, 0);
            if (m == MAP_FAILED) return 6;
            map = static_cast<const uint8_t*>(m);
        }
        bool ok = true;
        std::vector<bool> used(kStages, false);
        double dma_ms = 0;
        for (uint64_t r = 0; r < rounds && ok; ++r) {
            const int si = (int)(r % kStages);
            if (dma && used[si]) {
                (void)hipEventSynchronize(done[si]);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, beg[si], done[si]);
                dma_ms += ms;
            }
            const uint64_t a = r * C;
            std::vector<std::thread> pool;
            std::vector<char> tok(threads, 1);
            for (int t = 0; t < threads; ++t)
                pool.emplace_back([&, t] {
                    for (uint64_t i = (uint64_t)t; i < n; i += (uint64_t)threads) {
                        const uint64_t L = i == n - 1 ? total - (n - 1) * pl : pl;
                        if (a >= L) continue;
                        const uint64_t len = std::min<uint64_t>(C, L - a);
                        uint8_t* d = stage[si] + i * pitch;
                        const uint64_t off = i * pl + a;
                        if (mode == 0)
                            tok[t] &= pread_full(fd, d, (int64_t)off, (int64_t)len) ? 1 : 0;
                        else if (mode == 1)
                            std::memcpy(d, map + off, len);
                        else
                            copy_nt(d, map + off, len);
                    }
                    if (mode == 2) _mm_sfence();
                });
            for (auto& th : pool) th.join();
            for (char c : tok) ok = ok && c;
            if (dma) {
                (void)hipEventRecord(beg[si], ds);
                (void)hipMemcpyAsync(dev, stage[si], stage_bytes, hipMemcpyHostToDevice, ds);
                (void)hipEventRecord(done[si], ds);
                used[si] = true;
            }
        }
        if (dma) {
            (void)hipStreamSynchronize(ds);
            for (int k = 0; k < kStages; ++k) {
                // the last kStages rounds' copies (the loop above timed the earlier ones)
                if (!used[k]) continue;
                float ms = 0;
                (void)hipEventElapsedTime(&ms, beg[k], done[k]);
                dma_ms += ms;
            }
        }
        if (map) munmap(const_cast<uint8_t*>(map), total);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (!ok) return 7;
        rates.push_back(total / s / (double)(1ull << 30));
        busy.push_back(dma ? dma_ms * 1e-3 / s : 0);
    }
    std::vector<double> sr = rates;
    std::sort(sr.begin(), sr.end());
    const double med = sr[sr.size() / 2];
    std::printf("{\"mode\": %d, \"threads\": %d, \"chunk\": %llu, \"dma\": %d, \"populate\": %d, \"GiBps\": %.2f, "
                "\"runs\": [",
                mode, threads, (unsigned long long)C, (int)dma, (int)populate, med);
    for (size_t k = 0; k < rates.size(); ++k) std::printf("%s%.2f", k ? ", " : "", rates[k]);
    std::printf("], \"dma_busy\": [");
    for (size_t k = 0; k < busy.size(); ++k) std::printf("%s%.3f", k ? ", " : "", busy[k]);
    std::printf("]}\n");
    for (auto s : stage) (void)hipHostFree(s);
    if (dev) (void)hipFree(dev);
    close(fd);
    return 0;
}
