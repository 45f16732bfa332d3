// mmap_reg_probe.hip — can the bulk re-verify skip the pread copy?
//
// vx_verify_files preads every piece into a pinned stage and DMAs the stage:
// host memory is read twice and written once per byte.  The alternative maps
// the (page-cache warm) file, registers the mapping with hipHostRegister
// (read-only) and DMAs straight out of the page cache.  This times, for a
// file given on the command line: register the whole mapping, one flat H2D of
// it, unregister; and the same in windows of W MiB (register window k+1 while
// window k copies would overlap the two).  Prints one JSON line (ms, GiB/s).
// usage: mmap_reg_probe <file> [window_MiB...]
//        mmap_reg_probe <file> pipe <threads> <window_MiB>
//   pipe: fresh mapping, T threads register windows (window i on thread
//   i % T, in order) while the main thread DMAs each window as soon as it is
//   registered — the first-touch cost a single re-verify pass would pay.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const int fd = open(argv[1], O_RDONLY);
    if (fd < 0) return 3;
    struct stat st;
    fstat(fd, &st);
    const size_t bytes = st.st_size;
    // VX_POPULATE=0: map without pre-faulting (the file is page-cache warm but
    // not mapped, as a re-verify finds it); registration faults the pages in.
    const char* pe = std::getenv("VX_POPULATE");
    const int populate = (pe && pe[0] == '0') ? 0 : MAP_POPULATE;
    const double tm0 = now();
    void* m = mmap(nullptr, bytes, PROT_READ, MAP_SHARED | populate, fd, 0);
    const double tm1 = now();
    if (m == MAP_FAILED) return 4;
    uint8_t* d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) return 5;
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    std::string out = "{\"file_bytes\": " + std::to_string(bytes) + ", \"populate\": " + std::to_string(populate != 0);
    auto emit = [&](const std::string& k, double v) {
        char b[96];
        std::snprintf(b, sizeof b, ", \"%s\": %.3f", k.c_str(), v);
        out += b;
    };
    if (argc == 5 && std::string(argv[2]) == "pipe") {
        const int T = std::atoi(argv[3]);
        const size_t w = (size_t)std::atoi(argv[4]) << 20;
        const size_t nw = (bytes + w - 1) / w;
        std::vector<std::atomic<int>> ready(nw);
        for (auto& r : ready) r.store(0);
        const double t0 = now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                for (size_t i = t; i < nw; i += T) {
                    const size_t len = std::min(w, bytes - i * w);
                    const bool ok = hipHostRegister(static_cast<uint8_t*>(m) + i * w, len,
                                                    hipHostRegisterReadOnly) == hipSuccess;
                    ready[i].store(ok ? 1 : -1, std::memory_order_release);
                }
            });
        bool ok = true;
        for (size_t i = 0; i < nw; ++i) {
            int r;
            while ((r = ready[i].load(std::memory_order_acquire)) == 0) std::this_thread::yield();
            if (r < 0) ok = false;
            if (ok) (void)hipMemcpyAsync(d + i * w, static_cast<uint8_t*>(m) + i * w, std::min(w, bytes - i * w),
                                         hipMemcpyHostToDevice, s);
        }
        const double t1 = now();
        (void)hipStreamSynchronize(s);
        const double t2 = now();
        for (auto& x : th) x.join();
        emit("threads", T);
        emit("window_MiB", (double)(w >> 20));
        emit("ok", ok);
        emit("all_registered_ms", (t1 - t0) * 1e3);
        emit("total_ms", (t2 - t0) * 1e3);
        emit("GiBps", bytes / (t2 - t0) / (1 << 30));
        out += "}";
        std::printf("%s\n", out.c_str());
        return 0;
    }
    emit("mmap_ms", (tm1 - tm0) * 1e3);
    for (unsigned flags : {(unsigned)hipHostRegisterReadOnly, (unsigned)hipHostRegisterDefault}) {
        const std::string tag = flags ? "ro" : "default";
        for (int rep = 0; rep < 2; ++rep) {
            const double t0 = now();
            hipError_t e = hipHostRegister(m, bytes, flags);
            const double t1 = now();
            if (e != hipSuccess) {
                out += ", \"" + tag + "_error\": \"" + hipGetErrorString(e) + "\"";
                (void)hipGetLastError();
                break;
            }
            (void)hipMemcpyAsync(d, m, bytes, hipMemcpyHostToDevice, s);
            (void)hipStreamSynchronize(s);
            const double t2 = now();
            (void)hipHostUnregister(m);
            const double t3 = now();
            emit(tag + "_rep" + std::to_string(rep) + "_register_ms", (t1 - t0) * 1e3);
            if (rep == 1) {
                emit(tag + "_h2d_GiBps", bytes / (t2 - t1) / (1 << 30));
                emit(tag + "_unregister_ms", (t3 - t2) * 1e3);
                emit(tag + "_total_GiBps", bytes / (t3 - t0) / (1 << 30));
            }
        }
    }
    // windows: register all windows up front, then copy them in order (the
    // pipelined form would register window k+1 during window k's copy)
    for (int i = 2; i < argc; ++i) {
        const size_t w = (size_t)std::atoi(argv[i]) << 20;
        double reg = 0;
        const double t0 = now();
        bool ok = true;
        for (size_t o = 0; o < bytes && ok; o += w) {
            const size_t len = std::min(w, bytes - o);
            const double a = now();
            ok = hipHostRegister(static_cast<uint8_t*>(m) + o, len, hipHostRegisterReadOnly) == hipSuccess;
            reg += now() - a;
            if (ok) (void)hipMemcpyAsync(d + o, static_cast<uint8_t*>(m) + o, len, hipMemcpyHostToDevice, s);
        }
        (void)hipStreamSynchronize(s);
        const double t1 = now();
        for (size_t o = 0; o < bytes; o += w) (void)hipHostUnregister(static_cast<uint8_t*>(m) + o);
        if (!ok) {
            out += ", \"window_error\": 1";
            continue;
        }
        emit("win" + std::to_string(w >> 20) + "M_register_ms", reg * 1e3);
        emit("win" + std::to_string(w >> 20) + "M_GiBps", bytes / (t1 - t0) / (1 << 30));
    }
    out += "}";
    std::printf("%s\n", out.c_str());
    return 0;
}
