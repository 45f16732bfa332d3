// readers_stress.cpp — CPU test of vx_files::Readers (the pread pool behind
// vx_verify_files): many back-to-back run() generations whose item vector the
// caller rebuilds (and regrows) between runs; then the pipelined form
// verify_whole / verify_chunked use (start(g), check generation g-1's bytes
// while g reads into the other stage, wait(g); two item vectors alternating);
// then the queued form the re-verify uses since round 2 (submit() up to three
// jobs ahead, wait(ticket) in order with an occasional later ticket first,
// empty jobs mixed in, each job checked while later ones read), and the same
// with a zero-thread pool (reads inline in submit()); then whole-piece runs
// (vx_files::Runs) over a multi-file layout with an empty, a missing and a
// truncated file: every piece lands the concatenated bytes or is marked bad
// exactly when the per-piece walk would fail.
// Every item must land the right file bytes.  Built plain and with
// -fsanitize=thread by tests/test_native_cpu.py; exit 0 = ok.
//
// usage: readers_stress <scratch_file> [generations=3000] [threads=6]
#include <fcntl.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "vx_files.hpp"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const int gens = argc > 2 ? std::atoi(argv[2]) : 3000;
    const int nthreads = argc > 3 ? std::atoi(argv[3]) : 6;
    const uint32_t pl = 4096;
    const uint32_t npieces = 512;
    std::vector<uint8_t> file((size_t)pl * npieces);
    std::mt19937 rng(1);
    for (auto& b : file) b = (uint8_t)rng();
    FILE* f = std::fopen(argv[1], "wb");
    if (!f || std::fwrite(file.data(), 1, file.size(), f) != file.size()) return 2;
    std::fclose(f);
    const uint64_t len = file.size();
    const std::vector<vx_files::FileSpan> fs = vx_files::layout(&len, 1, pl);
    std::vector<int> fds{open(argv[1], O_RDONLY)};
    std::vector<uint8_t> bad(npieces, 0);
    std::vector<uint8_t> stage((size_t)pl * npieces);
    int errors = 0;
    {
        vx_files::Readers rd(nthreads, fs, fds, pl, bad.data(), 0);
        std::vector<vx_files::ReadItem> items;
        for (int g = 0; g < gens; ++g) {
            items.clear();
            items.shrink_to_fit();  // force a reallocation on every refill
            const uint32_t m = 1 + rng() % 64;
            const uint32_t base = rng() % (npieces - m);
            for (uint32_t k = 0; k < m; ++k) {
                const uint32_t p = base + k;
                const uint32_t a = rng() % 2 ? 0 : 1024;
                items.push_back(vx_files::ReadItem{stage.data() + (size_t)k * pl, p, a, pl - a});
            }
            rd.run(items);
            for (uint32_t k = 0; k < m; ++k) {
                const auto& it = items[k];
                if (std::memcmp(it.dst, file.data() + (size_t)it.piece * pl + it.start, it.len) != 0) ++errors;
            }
        }
        // pipelined: generation g reads into stage2[g & 1] from items2[g & 1]
        // while the caller checks generation g-1 (the other stage); a worker
        // still touching g-1's vector or stage after wait() would show here
        std::vector<vx_files::ReadItem> items2[2];
        std::vector<uint8_t> stage2[2] = {std::vector<uint8_t>((size_t)pl * 64), std::vector<uint8_t>((size_t)pl * 64)};
        auto check = [&](const std::vector<vx_files::ReadItem>& its) {
            for (const auto& it : its)
                if (std::memcmp(it.dst, file.data() + (size_t)it.piece * pl + it.start, it.len) != 0) ++errors;
        };
        for (int g = 0; g < gens; ++g) {
            auto& its = items2[g & 1];
            its.clear();
            its.shrink_to_fit();
            const uint32_t m = 1 + rng() % 64;
            const uint32_t base = rng() % (npieces - m);
            for (uint32_t k = 0; k < m; ++k) {
                const uint32_t a = rng() % 2 ? 0 : 2048;
                its.push_back(vx_files::ReadItem{stage2[g & 1].data() + (size_t)k * pl, base + k, a, pl - a});
            }
            rd.start(its);
            if (g > 0) check(items2[(g - 1) & 1]);  // the previous generation, during this one's reads
            rd.wait();
        }
        if (gens > 0) check(items2[(gens - 1) & 1]);

        // queued: a ring of 4 jobs, up to 3 in flight past the one awaited
        auto queued = [&](vx_files::Readers& r, int njobs) {
            constexpr int K = 4;
            std::vector<vx_files::ReadItem> ring[K];
            std::vector<uint8_t> st[K];
            uint64_t ticket[K] = {};
            for (auto& v : st) v.resize((size_t)pl * 64);
            int next = 0;
            for (int g = 0; g < njobs; ++g) {
                for (; next < njobs && next <= g + K - 1; ++next) {
                    auto& its = ring[next % K];
                    its.clear();
                    its.shrink_to_fit();
                    const uint32_t m = rng() % 8 == 0 ? 0 : 1 + rng() % 64;  // some empty jobs
                    const uint32_t base = rng() % (npieces - 64);
                    for (uint32_t k = 0; k < m; ++k) {
                        const uint32_t a = (uint32_t)(rng() % 4) * 512;
                        its.push_back(vx_files::ReadItem{st[next % K].data() + (size_t)k * pl, base + k, a, pl - a});
                    }
                    ticket[next % K] = r.submit(its);
                }
                if (g + 1 < next && rng() % 5 == 0) r.wait(ticket[(g + 1) % K]);  // a later job first
                r.wait(ticket[g % K]);
                check(ring[g % K]);
            }
            r.wait();
        };
        queued(rd, gens);
        vx_files::Readers inline_rd(0, fs, fds, pl, bad.data(), 0);
        queued(inline_rd, 200);
    }
    close(fds[0]);
    for (uint8_t b : bad) errors += b;

    {  // coalesced runs over several files
        const uint32_t rpl = 1024;
        const std::string base = std::string(argv[1]) + ".mf";
        // declared lengths; file 3 is never created (missing), file 5 is written 3000 bytes short
        const std::vector<uint64_t> flen{3 * rpl + 100, 0, 5 * rpl - 100, 9 * rpl, 2 * rpl + 500, 40 * rpl + 37};
        const size_t missing = 3, truncated = 5, cut = 3000;
        std::vector<uint8_t> all;
        std::vector<int> mfds;
        for (size_t f = 0; f < flen.size(); ++f) {
            std::vector<uint8_t> d(flen[f]);
            for (auto& b : d) b = (uint8_t)rng();
            all.insert(all.end(), d.begin(), d.end());
            const std::string path = base + std::to_string(f);
            if (f != missing) {
                FILE* g = std::fopen(path.c_str(), "wb");
                const size_t w = f == truncated ? d.size() - cut : d.size();
                if (!g || (w && std::fwrite(d.data(), 1, w, g) != w)) return 2;
                std::fclose(g);
            }
            mfds.push_back(open(path.c_str(), O_RDONLY));
        }
        const std::vector<vx_files::FileSpan> mfs = vx_files::layout(flen.data(), flen.size(), rpl);
        const uint64_t total = all.size(), n = (total + rpl - 1) / rpl;
        std::vector<uint64_t> fstart{0};
        for (uint64_t L : flen) fstart.push_back(fstart.back() + L);
        for (uint64_t max_bytes : {(uint64_t)0, (uint64_t)4 * rpl, (uint64_t)1 << 20}) {
            std::vector<uint8_t> mbad(n, 0), st(n * rpl, 0);
            std::vector<vx_files::ReadItem> its;
            {
                vx_files::Readers r(3, mfs, mfds, rpl, mbad.data(), 0);
                vx_files::Runs runs = r.runs(max_bytes);
                for (uint64_t i = 0; i < n; ++i) runs.add(its, st.data() + i * rpl, i, std::min<uint64_t>(rpl, total - i * rpl));
                r.wait(r.submit(its));
            }
            if (max_bytes >= (1u << 20) && its.size() >= n / 2) ++errors;  // runs did not coalesce
            for (uint64_t i = 0; i < n; ++i) {
                const uint64_t a = i * rpl, b = std::min<uint64_t>(total, a + rpl);
                bool fails = false;  // the walk fails if the piece touches the missing file or the cut tail
                for (size_t f = 0; f < flen.size(); ++f) {
                    const uint64_t lo = std::max(a, fstart[f]), hi = std::min(b, fstart[f + 1]);
                    if (lo >= hi) continue;
                    if (f == missing) fails = true;
                    if (f == truncated && hi > fstart[f + 1] - cut) fails = true;
                }
                if (fails != (mbad[i] != 0)) ++errors;
                if (!fails && std::memcmp(st.data() + a, all.data() + a, b - a) != 0) ++errors;
            }
        }
        for (size_t f = 0; f < flen.size(); ++f) {
            if (mfds[f] >= 0) close(mfds[f]);
            std::remove((base + std::to_string(f)).c_str());
        }
    }
    std::printf("{\"generations\": %d, \"errors\": %d}\n", gens, errors);
    return errors == 0 ? 0 : 1;
}
