// pread_probe.hip — host-side ceiling of the bulk re-verify reader: T threads
// pread 256 KiB chunks of a (page-cache warm) file into a hipHostMalloc'd
// stage, as vx_files::Readers does, with no GPU work.  Prints one JSON line.
// usage: pread_probe <file> [threads...]
// VX_DMA=1: one more thread streams 512 MiB H2D copies out of a second pinned
// buffer the whole time (the re-verify's DMA competing for host memory);
// the DMA rate over the read window is reported beside the read rate.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
    const char* de = std::getenv("VX_DMA");
    const bool dma = de && de[0] == '1';
    uint8_t *src = nullptr, *dev = nullptr;
    hipStream_t ds = nullptr;
    if (dma && (hipHostMalloc(&src, stage, hipHostMallocDefault) != hipSuccess ||
                hipMalloc(&dev, stage) != hipSuccess || hipStreamCreate(&ds) != hipSuccess))
        return 5;
    if (dma) std::memset(src, 1, stage);
    std::printf("{\"file_bytes\": %zu, \"dma\": %d", bytes, (int)dma);
    for (int T : ts) {
        double best = 0, best_dma = 0;
        for (int rep = 0; rep < 3; ++rep) {
            std::atomic<size_t> next{0};
            std::atomic<bool> stop{false};
            std::atomic<size_t> moved{0};
            std::thread dt;
            if (dma)
                dt = std::thread([&] {
                    const size_t dc = 64ull << 20;  // 1.2 ms per copy: fine-grained count
                    for (size_t o = 0; !stop.load(); o = (o + dc) % stage) {
                        (void)hipMemcpyAsync(dev + o, src + o, dc, hipMemcpyHostToDevice, ds);
                        (void)hipStreamSynchronize(ds);
                        if (!stop.load()) moved += dc;
                    }
                });
            if (dma) std::this_thread::sleep_for(std::chrono::milliseconds(30));  // DMA in flight
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
            const size_t m0 = moved.load();
            for (auto& x : th) x.join();
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            const size_t m1 = moved.load();
            stop = true;
            if (dt.joinable()) dt.join();
            if (bytes / s / (1 << 30) > best) {
                best = bytes / s / (1 << 30);
                best_dma = (m1 - m0) / s / (1 << 30);
            }
        }
        std::printf(", \"pread_GiBps_t%d\": %.2f", T, best);
        if (dma) std::printf(", \"dma_GiBps_t%d\": %.2f", T, best_dma);
    }
    std::printf("}\n");
    (void)hipHostFree(buf);
    close(fd);
    return 0;
}
