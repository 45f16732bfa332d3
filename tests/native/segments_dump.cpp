// segments_dump.cpp — CPU harness for the re-verify's piece -> file-segment
// mapping (vortex_amd/csrc/vx_files.hpp: layout + segments), used by
// tests/test_native_cpu.py.  Not the product; no GPU.
//
// stdin: the torrent's file lengths, one per line.  argv: piece_length
// [check_every].  stdout: one line per piece, "f off len" triples separated by
// ';' (the engine's segments), then a JSON summary line.  With check_every = k
// > 0, every k-th piece is also mapped by the reference's own form of the walk
// — every file of the torrent filtered by start_piece <= idx <= end_piece
// (file_store.rs:238-241), segments as at file_store.rs:245-269 — and any
// difference is counted in "linear_mismatches".
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "vx_files.hpp"

static void linear_walk(const std::vector<vx_files::FileSpan>& fs, int64_t piece, uint32_t pl,
                        std::vector<vx_files::Seg>& out) {
    out.clear();
    int64_t total = 0;
    for (size_t f = 0; f < fs.size(); ++f) {
        const vx_files::FileSpan& s = fs[f];
        if (!(s.start_piece <= piece && piece <= s.end_piece)) continue;
        const int64_t off = (piece - s.start_piece) * (int64_t)pl - s.start_offset + total;
        const int64_t to_read =
            piece == s.end_piece ? s.end_offset - total : std::min<int64_t>((int64_t)pl - total, s.len);
        if (to_read <= 0) continue;
        out.push_back(vx_files::Seg{(uint32_t)f, off, to_read});
        total += to_read;
    }
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: segments_dump piece_length [check_every] < lengths\n");
        return 2;
    }
    const uint32_t pl = (uint32_t)std::strtoul(argv[1], nullptr, 0);
    const long check_every = argc > 2 ? std::strtol(argv[2], nullptr, 0) : 0;
    std::vector<uint64_t> lens;
    unsigned long long x;
    while (std::scanf("%llu", &x) == 1) lens.push_back(x);
    uint64_t total = 0;
    for (uint64_t L : lens) total += L;
    const int64_t n = pl ? (int64_t)((total + pl - 1) / pl) : 0;

    const auto t0 = std::chrono::steady_clock::now();
    const auto fs = vx_files::layout(lens.data(), lens.size(), pl);
    std::vector<std::vector<vx_files::Seg>> all((size_t)n);
    for (int64_t p = 0; p < n; ++p) vx_files::segments(fs, p, pl, all[(size_t)p]);
    const double build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();

    long mism = 0, checked = 0;
    if (check_every > 0) {
        std::vector<vx_files::Seg> ref;
        for (int64_t p = 0; p < n; p += check_every) {
            linear_walk(fs, p, pl, ref);
            ++checked;
            const auto& got = all[(size_t)p];
            bool same = ref.size() == got.size();
            for (size_t k = 0; same && k < ref.size(); ++k)
                same = ref[k].file == got[k].file && ref[k].off == got[k].off && ref[k].len == got[k].len;
            mism += !same;
        }
    }
    std::string line;
    for (int64_t p = 0; p < n; ++p) {
        line.clear();
        for (size_t k = 0; k < all[(size_t)p].size(); ++k) {
            const auto& s = all[(size_t)p][k];
            if (k) line += ';';
            line += std::to_string(s.file) + ' ' + std::to_string(s.off) + ' ' + std::to_string(s.len);
        }
        std::puts(line.c_str());
    }
    std::printf("{\"files\": %zu, \"pieces\": %lld, \"build_ms\": %.3f, \"linear_checked\": %ld, "
                "\"linear_mismatches\": %ld}\n",
                lens.size(), (long long)n, build_ms, checked, mism);
    return 0;
}
