// direct_check.cpp — CPU harness for vx_files::DirectIo (O_DIRECT reads of
// ranges that are not in the page cache), used by tests/test_native_cpu.py.
// Not the product; no GPU.
//
// argv: path mode [replacement | big].  mode 1 = DirectIo enabled, 0 =
// disabled.  With a replacement path, that file is renamed over `path` after
// `path` was opened and before DirectIo is built: every read must still return
// the opened file's bytes (the O_DIRECT descriptor reopens the open file, not
// the path).  mode 2 = enabled, with `big` listed as the torrent's first file
// before `path`, so `path` is a small share of the torrent's bytes (its
// residency gets the per-file minimum of samples).  Reads a fixed list of ranges of the file — 4 KiB aligned
// and not, aligned and unaligned destinations, a range ending at EOF, an
// aligned head with an unaligned tail — through DirectIo::read into a
// page-aligned buffer, and compares each with a plain buffered pread.  Prints
// {"reads": n, "mismatches": k, "direct_bytes": b, "resident": f}, f being
// DirectIo::resident_fraction() sampled before any read.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "vx_files.hpp"

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: direct_check path mode [replacement]\n");
        return 2;
    }
    const char* path = argv[1];
    const int mode = std::atoi(argv[2]);
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    struct stat st;
    if (fd < 0 || fstat(fd, &st) != 0) return 2;
    const int64_t size = st.st_size;
    std::vector<int> fds{fd};
    uint32_t fi = 0;  // this file's index in the torrent
    if (mode == 2) {
        const int big = argc > 3 ? open(argv[3], O_RDONLY | O_CLOEXEC) : -1;
        if (big < 0) return 2;
        fds = {big, fd};
        fi = 1;
    } else if (argc > 3 && rename(argv[3], path) != 0) {  // the path now names another file
        return 2;
    }
    vx_files::DirectIo dio(fds, mode != 0);
    const double resident = dio.resident_fraction();
    const int64_t K = 4096;
    struct R {
        int64_t off, len, dst_skew;
    };
    const std::vector<R> ranges = {
        {0, 4 * K, 0},           {K, 64 * K, 0},          {3 * K, 5 * K + 100, 0}, {100, 8 * K, 0},
        {2 * K, 16 * K, 16},     {size - 8 * K, 8 * K, 0}, {size - 3 * K - 7, 3 * K + 7, 0},
        {16 * K, 256 * K, 0},    {size / 2 & ~(K - 1), 300 * K + 1, 0}, {5 * K, K - 1, 0},
        {size / 8 * 7 & ~(K - 1), 64 * K, 0},  // aligned, in the last eighth
    };
    uint8_t* a = nullptr;
    if (posix_memalign(reinterpret_cast<void**>(&a), K, (size_t)size + 2 * K) != 0) return 2;
    std::vector<uint8_t> b((size_t)size + 2 * K);
    int mism = 0, n = 0;
    for (const R& r : ranges) {
        if (r.off < 0 || r.off + r.len > size) continue;
        ++n;
        std::memset(a, 0xAB, (size_t)r.len + r.dst_skew);
        const bool ok = dio.read(fi, fd, a + r.dst_skew, r.off, r.len);
        const bool okb = vx_files::read_full(fd, b.data(), r.off, r.len);
        if (!ok || !okb || std::memcmp(a + r.dst_skew, b.data(), (size_t)r.len) != 0) ++mism;
    }
    std::printf("{\"reads\": %d, \"mismatches\": %d, \"direct_bytes\": %llu, \"resident\": %.4f}\n", n, mism,
                (unsigned long long)dio.direct_bytes(), resident);
    free(a);
    for (int d : fds) close(d);
    return 0;
}
