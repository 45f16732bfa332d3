// readers_probe.cpp — the re-verify's read side alone:
// vx_files::Readers reading a file in the resumable rounds of
// vx_verify_files (chunk k of every piece of the window per round, into
// pinned stages used round-robin, up to `ahead` rounds queued), with no GPU
// work, optionally with the DirectIo residency probe, and optionally with one
// thread streaming each finished round's stage to the GPU (hipMemcpyAsync, as
// the pipeline's copy chain does).  Tells whether the readers bind by
// themselves or only inside the full pipeline.
//
// usage: readers_probe <file> <piece_len> [threads=16] [chunk=262144] [ahead=2] [stages=4] [dio=1] [dma=0] [reps=3] [evict=0] [mem=0]
//   evict=1: drop the file's pages (fsync + POSIX_FADV_DONTNEED) before every rep (a cold re-verify)
//   mem: the stages' memory, 0 hipHostMalloc (the engine's), 1 plain mmap (not pinned), 2 mmap + hipHostRegister,
//        3 / 4 as 1 / 2 with MADV_HUGEPAGE (2 MiB pages where THP allows)
// Prints one JSON line: best GiB/s over reps, the readers' own rate (bytes /
// summed pread time) and, with dma, the copy rate.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <thread>
#include <vector>

#include "vx_files.hpp"

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const char* path = argv[1];
    const uint32_t pl = (uint32_t)std::strtoul(argv[2], nullptr, 0);
    const int threads = argc > 3 ? std::atoi(argv[3]) : 16;
    const uint64_t C = argc > 4 ? std::strtoull(argv[4], nullptr, 0) : 262144;
    const size_t ahead = argc > 5 ? (size_t)std::atoi(argv[5]) : 2;
    const int nst = argc > 6 ? std::atoi(argv[6]) : 4;
    const bool use_dio = argc > 7 ? std::atoi(argv[7]) != 0 : true;
    const bool dma = argc > 8 ? std::atoi(argv[8]) != 0 : false;
    const int reps = argc > 9 ? std::atoi(argv[9]) : 3;
    const bool evict = argc > 10 ? std::atoi(argv[10]) != 0 : false;
    const int mem = argc > 11 ? std::atoi(argv[11]) : 0;
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    struct stat st;
    if (fd < 0 || fstat(fd, &st) != 0) return 3;
    const uint64_t total = (uint64_t)st.st_size;
    const uint64_t n = (total + pl - 1) / pl;
    const uint64_t last_len = total - (n - 1) * pl;
    const uint64_t pitch = (C + 4095) / 4096 * 4096;
    const uint64_t stage_bytes = n * pitch;
    std::vector<uint8_t*> stage(nst, nullptr);
    for (auto& s : stage) {
        if (mem == 0) {
            if (hipHostMalloc(&s, stage_bytes, hipHostMallocDefault) != hipSuccess) return 4;
            continue;
        }
        const bool huge = mem >= 3;
        void* p = mmap(nullptr, stage_bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | (huge ? 0 : MAP_POPULATE),
                       -1, 0);
        if (p == MAP_FAILED) return 4;
        s = static_cast<uint8_t*>(p);
        if (huge) {
            (void)madvise(s, stage_bytes, MADV_HUGEPAGE);
            for (uint64_t o = 0; o < stage_bytes; o += 4096) s[o] = 0;
        }
        if ((mem == 2 || mem == 4) && hipHostRegister(s, stage_bytes, hipHostRegisterDefault) != hipSuccess) return 4;
    }
    uint8_t* dev = nullptr;
    hipStream_t ds = nullptr;
    if (dma && (hipMalloc(&dev, stage_bytes) != hipSuccess || hipStreamCreate(&ds) != hipSuccess)) return 5;
    std::vector<int> fds{fd};
    const uint64_t lens[1] = {total};
    const auto fs = vx_files::layout(lens, 1, pl);
    double best = 0, best_own = 0, best_copy = 0;
    for (int rep = 0; rep < reps; ++rep) {
        if (evict) {
            (void)fsync(fd);
            (void)posix_fadvise(fd, 0, 0, POSIX_FADV_DONTNEED);
        }
        std::vector<uint8_t> bad(n, 0);
        const vx_files::DirectIo dio(fds, use_dio);
        vx_files::Readers rd(threads, fs, fds, pl, bad.data(), 0, use_dio ? &dio : nullptr);
        std::vector<std::vector<vx_files::ReadItem>> items(nst);
        std::deque<std::pair<int, uint64_t>> q;  // (stage, ticket)
        std::vector<uint64_t> round_bytes(nst, 0);
        double copy_s = 0;
        uint64_t copied = 0;
        const auto t0 = std::chrono::steady_clock::now();
        const uint64_t rounds = (pl + C - 1) / C;
        uint64_t next = 0;
        int si = 0;
        auto finish_one = [&] {
            const auto h = q.front();
            q.pop_front();
            rd.wait(h.second);
            if (dma) {  // the copy chain: one H2D of the round, waited for before its stage is reused
                const auto c0 = std::chrono::steady_clock::now();
                (void)hipMemcpyAsync(dev, stage[h.first], round_bytes[h.first], hipMemcpyHostToDevice, ds);
                (void)hipStreamSynchronize(ds);
                copy_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count();
                copied += round_bytes[h.first];
            }
        };
        while (next < rounds || !q.empty()) {
            while (next < rounds && q.size() <= ahead) {
                auto& it = items[si];
                it.clear();
                const uint64_t a = next * C;
                uint64_t m = 0;
                for (uint64_t i = 0; i < n; ++i) {
                    const uint64_t L = i == n - 1 ? last_len : pl;
                    if (a >= L) continue;
                    it.push_back(vx_files::ReadItem{stage[si] + m * pitch, i, a, std::min<uint64_t>(C, L - a)});
                    ++m;
                }
                round_bytes[si] = m ? (m - 1) * pitch + it.back().len : 0;
                q.emplace_back(si, rd.submit(it));
                si = (si + 1) % nst;
                ++next;
            }
            finish_one();
        }
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (uint8_t b : bad)
            if (b) return 6;
        const double gib = (double)(1ull << 30);
        if (total / s / gib > best) {
            best = total / s / gib;
            best_own = rd.busy_ns() ? rd.bytes_read() / (rd.busy_ns() * 1e-9) / gib : 0;
            best_copy = copy_s > 0 ? copied / copy_s / gib : 0;
        }
    }
    std::printf("{\"threads\": %d, \"chunk\": %llu, \"ahead\": %zu, \"stages\": %d, \"dio\": %d, \"dma\": %d, "
                "\"evict\": %d, \"mem\": %d, \"GiBps\": %.2f, \"reader_own_GiBps_per_thread\": %.2f, "
                "\"copy_GiBps\": %.2f}\n",
                threads, (unsigned long long)C, ahead, nst, (int)use_dio, (int)dma, (int)evict, mem, best, best_own,
                best_copy);
    for (auto s : stage) {
        if (mem == 0) {
            (void)hipHostFree(s);
            continue;
        }
        if (mem == 2 || mem == 4) (void)hipHostUnregister(s);
        munmap(s, stage_bytes);
    }
    if (dev) (void)hipFree(dev);
    close(fd);
    return 0;
}
