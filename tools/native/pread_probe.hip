// pread_probe.hip — host-side ceiling of the bulk re-verify reader: T threads
// pread chunks of a (page-cache warm) file into a hipHostMalloc'd stage, as
// vx_files::Readers does, with no GPU work.  Prints one JSON line.
// usage: pread_probe <file> [threads...] [c=<chunk bytes>...] [p=<piece bytes>] [dma]
//   c=   read sizes to try (default 262144)
//   p=   chunk-major order inside pieces of this size, as the re-verify's
//        resumable rounds read (chunk k of every piece, then chunk k+1; 0 =
//        the file in order, default)
//   dma  one more thread streams 512 MiB H2D copies out of a second pinned
//        buffer the whole time (the re-verify's DMA competing for host
//        memory); the DMA rate over the read window is reported beside.
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
    const size_t bytes = st.st_size, chunk = 256 * 1024;  // default read size
    const size_t stage = 512ull << 20;  // one slot's stage, reused round-robin
    uint8_t* buf = nullptr;
    if (hipHostMalloc(&buf, stage, hipHostMallocDefault) != hipSuccess) return 4;
    std::vector<int> ts;
    std::vector<size_t> chunks;
    size_t piece = 0;
    bool dma = false;
    for (int i = 2; i < argc; ++i) {
        if (argv[i][0] == 'c' && argv[i][1] == '=') chunks.push_back(std::strtoull(argv[i] + 2, nullptr, 0));
        else if (argv[i][0] == 'p' && argv[i][1] == '=') piece = std::strtoull(argv[i] + 2, nullptr, 0);
        else if (std::strcmp(argv[i], "dma") == 0) dma = true;
        else ts.push_back(std::atoi(argv[i]));
    }
    if (ts.empty()) ts = {1, 4, 8, 16};
    if (chunks.empty()) chunks = {chunk};
    uint8_t *src = nullptr, *dev = nullptr;
    hipStream_t ds = nullptr;
    if (dma && (hipHostMalloc(&src, stage, hipHostMallocDefault) != hipSuccess ||
                hipMalloc(&dev, stage) != hipSuccess || hipStreamCreate(&ds) != hipSuccess))
        return 5;
    if (dma) std::memset(src, 1, stage);
    std::printf("{\"file_bytes\": %zu, \"dma\": %d, \"piece\": %zu", bytes, (int)dma, piece);
    for (const size_t C : chunks)
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
                    // chunk-major inside pieces: item k is chunk k / npieces of piece k % npieces
                    const size_t per = piece && piece > C ? piece / C : 1, npieces = piece ? (bytes + piece - 1) / piece : 0;
                    for (;;) {
                        const size_t k = next.fetch_add(1);
                        size_t off = k * C;
                        if (per > 1) {
                            const size_t r = k / npieces, pc = k % npieces;
                            if (r >= per) return;
                            off = pc * piece + r * C;
                        }
                        if (off >= bytes) {
                            if (per > 1) continue;
                            return;
                        }
                        const size_t len = std::min(C, bytes - off);
                        if (pread(fd, buf + (k * C % stage), len, (off_t)off) != (ssize_t)len) std::abort();
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
        std::printf(", \"pread_GiBps_c%zu_t%d\": %.2f", C, T, best);
        if (dma) std::printf(", \"dma_GiBps_c%zu_t%d\": %.2f", C, T, best_dma);
    }
    std::printf("}\n");
    (void)hipHostFree(buf);
    close(fd);
    return 0;
}
