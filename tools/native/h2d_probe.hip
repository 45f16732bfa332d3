// h2d_probe.hip — PCIe H2D microbenchmark for the host engine's copy policy:
// hipHostMalloc'd vs hipHostRegister'd (mmap) sources, one copy vs chunked,
// one stream vs several.  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstring>
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
    uint8_t* hm = nullptr;
    CK(hipHostMalloc(&hm, bytes, hipHostMallocDefault));
    std::memset(hm, 1, bytes);
    uint8_t* mm = static_cast<uint8_t*>(mmap(nullptr, bytes, PROT_READ | PROT_WRITE,
                                              MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0));
    std::memset(mm, 1, bytes);
    CK(hipHostRegister(mm, bytes, hipHostRegisterDefault));
    std::vector<hipStream_t> st(8);
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::printf("{");
    const char* names[2] = {"hostmalloc", "registered"};
    uint8_t* srcs[2] = {hm, mm};
    bool first = true;
    for (int si = 0; si < 2; ++si) {
        for (int chunks : {1, 8, 64}) {
            for (int nst : {1, 2, 4, 8}) {
                if (chunks == 1 && nst > 1) continue;
                double best = 0;
                for (int rep = 0; rep < 3; ++rep) {
                    CK(hipDeviceSynchronize());
                    const double t0 = now();
                    const size_t cb = bytes / chunks;
                    for (int c = 0; c < chunks; ++c)
                        CK(hipMemcpyAsync(d + c * cb, srcs[si] + c * cb, cb, hipMemcpyHostToDevice, st[c % nst]));
                    CK(hipDeviceSynchronize());
                    const double gbs = bytes / (now() - t0) / (1 << 30);
                    if (gbs > best) best = gbs;
                }
                std::printf("%s\"%s_c%d_s%d\": %.2f", first ? "" : ", ", names[si], chunks, nst, best);
                first = false;
            }
        }
    }
    std::printf("}\n");
    CK(hipHostUnregister(mm));
    munmap(mm, bytes);
    CK(hipHostFree(hm));
    CK(hipFree(d));
    return 0;
}
