// pread_probe.hip — host-side ceiling of the bulk re-verify reader: T threads
// pread 256 KiB chunks of a (page-cache warm) file into a hipHostMalloc'd
// stage, as vx_files::Readers does, with no GPU work.  Prints one JSON line.
// usage: pread_probe <file> [threads...]
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const int fd = open(argv[1], O_RDONLY);
    if (fd < 0) return 3;
    struct stat st;
    fstat(fd, &st);
    const size_t bytes = st.st_size, chunk = 256 * 1024;
    const size_t stage = 512ull << 20;  // one slot's stage, reused round-robin
    uint8_t* buf = nullptr;
    if (hipHostMalloc(&buf, stage, hipHostMallocDefault) != hipSuccess) return 4;
    std::vector<int> ts;
    for (int i = 2; i < argc; ++i) ts.push_back(std::atoi(argv[i]));
    if (ts.empty()) ts = {1, 4, 8, 16};
    std::printf("{\"file_bytes\": %zu", bytes);
    for (int T : ts) {
        double best = 0;
        for (int rep = 0; rep < 3; ++rep) {
            std::atomic<size_t> next{0};
            const auto t0 = std::chrono::steady_clock::now();
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t)
                th.emplace_back([&] {
                    for (;;) {
                        const size_t k = next.fetch_add(1);
                        const size_t off = k * chunk;
                        if (off >= bytes) return;
                        const size_t len = std::min(chunk, bytes - off);
                        if (pread(fd, buf + (off % stage), len, (off_t)off) != (ssize_t)len) std::abort();
                    }
                });
            for (auto& x : th) x.join();
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            best = std::max(best, bytes / s / (1 << 30));
        }
        std::printf(", \"pread_GiBps_t%d\": %.2f", T, best);
    }
    std::printf("}\n");
    (void)hipHostFree(buf);
    close(fd);
    return 0;
}
