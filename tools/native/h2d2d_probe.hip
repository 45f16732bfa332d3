// h2d2d_probe.hip — can the host engine move pieces chunk-major over PCIe?
//
// The chunked batch path sends chunk k of every piece of a
// window before chunk k+1.  With the pieces strided in a registered host
// buffer that is one hipMemcpy2DAsync per round (width = chunk, height =
// pieces, source pitch = piece stride); otherwise it is one hipMemcpyAsync
// per piece chunk.  This measures both against one flat copy of the same
// bytes.  Prints one JSON line (GiB/s, best of 3).
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstring>
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

int main() {
    const size_t bytes = 2ull << 30;
    uint8_t* d = nullptr;
    CK(hipMalloc(&d, bytes));
    uint8_t* mm = static_cast<uint8_t*>(mmap(nullptr, bytes, PROT_READ | PROT_WRITE,
                                              MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0));
    std::memset(mm, 1, bytes);
    CK(hipHostRegister(mm, bytes, hipHostRegisterDefault));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::string out = "{";
    auto emit = [&](const std::string& k, double v) {
        char b[96];
        std::snprintf(b, sizeof b, "%s\"%s\": %.2f", out.size() > 1 ? ", " : "", k.c_str(), v);
        out += b;
    };
    // warm the copy path
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
        emit("flat", best);
    }
    for (size_t pl : {size_t(256) << 10, size_t(2) << 20}) {
        const size_t n = bytes / pl;
        for (size_t C : {size_t(32) << 10, size_t(64) << 10, size_t(128) << 10, size_t(256) << 10}) {
            if (C > pl) continue;
            const size_t rounds = pl / C;
            double best2d = 0, best1d = 0;
            for (int rep = 0; rep < 3; ++rep) {
                double t0 = now();
                for (size_t k = 0; k < rounds; ++k)
                    CK(hipMemcpy2DAsync(d + k * C, pl, mm + k * C, pl, C, n, hipMemcpyHostToDevice, st));
                CK(hipStreamSynchronize(st));
                best2d = std::max(best2d, bytes / (now() - t0) / (1 << 30));
                if (n * rounds > 16384) continue;  // per-chunk copies only where the call count is sane
                t0 = now();
                for (size_t k = 0; k < rounds; ++k)
                    for (size_t i = 0; i < n; ++i)
                        CK(hipMemcpyAsync(d + i * pl + k * C, mm + i * pl + k * C, C, hipMemcpyHostToDevice, st));
                CK(hipStreamSynchronize(st));
                best1d = std::max(best1d, bytes / (now() - t0) / (1 << 30));
            }
            const std::string tag = "pl" + std::to_string(pl >> 10) + "K_c" + std::to_string(C >> 10) + "K";
            emit("2d_" + tag, best2d);
            if (best1d > 0) emit("percopy_" + tag, best1d);
        }
    }
    out += "}";
    std::printf("%s\n", out.c_str());
    CK(hipHostUnregister(mm));
    munmap(mm, bytes);
    CK(hipFree(d));
    return 0;
}
