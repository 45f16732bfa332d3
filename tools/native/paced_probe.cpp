// paced_probe.cpp — the download path at network-realistic arrival rates: what
// the engine costs vortex's event-loop thread, and how long a piece waits for
// its verdict.
//
// vortex hashes a piece when its last subpiece arrives (scope.spawn,
// peer_connection.rs:1145-1158) and drains the verdicts once per loop turn
// (downloaded_piece_rc.try_recv, torrent.rs:415-442, called at
// event_loop.rs:554-557); the loop waits at most 150 ms per turn for CQEs
// (event_loop.rs:438-439) and spawn never blocks.  This models that loop:
// pieces "arrive" at `rate` GB/s into buffers of a BufferPool (one registered
// mmap per buffer, buf_pool.rs:92-98); every `tick_us` a turn submits the
// pieces that arrived since the last turn (vx_submit), calls vx_flush once,
// and polls (vx_poll), returning each completed piece's buffer to the pool.
// A piece that arrives while every buffer is still being hashed waits for a
// buffer (the socket would simply not be read: counted as pool_waits).
//
// Prints one JSON line: the achieved rate, the loop thread's time inside
// vx_submit / vx_flush / vx_poll per second of wall time, the longest single
// call, the engine's own submit_stall (vx_stats), and submit-to-poll latency
// percentiles of every piece.  Every verdict must match.
//
// usage: paced_probe <piece_len> <rate_GBps> [seconds=1.5] [tick_us=1000] [nbuf=8192] [slots=4]
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "vx_hash.h"

using clk = std::chrono::steady_clock;

static double since(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

static double pct(std::vector<double>& v, double p) {
    if (v.empty()) return 0.0;
    const size_t k = std::min(v.size() - 1, (size_t)(p * (double)(v.size() - 1) + 0.5));
    std::nth_element(v.begin(), v.begin() + (long)k, v.end());
    return v[k];
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s piece_len rate_GBps [seconds] [tick_us] [nbuf] [slots]\n", argv[0]);
        return 2;
    }
    const uint32_t plen = (uint32_t)std::strtoul(argv[1], nullptr, 0);
    const double rate = std::atof(argv[2]) * 1e9;  // bytes per second
    const double seconds = argc > 3 ? std::atof(argv[3]) : 1.5;
    const double tick = (argc > 4 ? std::atof(argv[4]) : 1000.0) * 1e-6;
    const uint32_t nbuf = argc > 5 ? (uint32_t)std::atoi(argv[5]) : 8192;
    vx_config cfg;
    vx_config_default(&cfg, plen);
    if (argc > 6) cfg.slots = (uint32_t)std::atoi(argv[6]);
    vx_ctx* ctx = nullptr;
    if (int rc = vx_create(&cfg, &ctx)) {
        std::fprintf(stderr, "vx_create: %d %s\n", rc, vx_last_error());
        return 1;
    }
    std::vector<uint8_t*> bufs(nbuf);
    std::vector<const uint8_t*> ptrs(nbuf);
    std::vector<uint32_t> lens(nbuf, plen);
    std::mt19937_64 rng(plen ^ 0x9ACED);
    for (uint32_t b = 0; b < nbuf; ++b) {
        void* m = mmap(nullptr, plen, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
        if (m == MAP_FAILED) return 1;
        bufs[b] = static_cast<uint8_t*>(m);
        ptrs[b] = bufs[b];
        for (size_t i = 0; i < plen / 8; ++i) reinterpret_cast<uint64_t*>(bufs[b])[i] = rng();
        if (int rc = vx_register_host_buffer(ctx, bufs[b], plen)) {
            std::fprintf(stderr, "register: %d %s\n", rc, vx_last_error());
            return 1;
        }
    }
    std::vector<uint8_t> digests((size_t)nbuf * 20);
    if (int rc = vx_sha1_batch(ctx, ptrs.data(), lens.data(), nbuf, digests.data())) {
        std::fprintf(stderr, "vx_sha1_batch: %d %s\n", rc, vx_last_error());
        return 1;
    }
    for (uint32_t b = 0; b < nbuf; b += 97) digests[(size_t)b * 20 + 3] ^= 1;  // planted mismatches
    std::vector<uint32_t> free_bufs(nbuf);
    for (uint32_t b = 0; b < nbuf; ++b) free_bufs[b] = nbuf - 1 - b;
    std::shuffle(free_bufs.begin(), free_bufs.end(), rng);
    std::vector<clk::time_point> t_sub(nbuf);
    std::vector<double> lat;
    lat.reserve(1 << 20);
    std::vector<vx_completion> cq(4096);
    uint64_t submitted = 0, polled = 0, wrong = 0, pool_waits = 0, turns = 0, late_turns = 0;
    double call_s = 0, max_call = 0, submit_s = 0, flush_s = 0, poll_s = 0;
    auto timed = [&](auto&& fn, double& acc) -> int {
        const auto a = clk::now();
        const int rc = fn();
        const double d = since(a, clk::now());
        acc += d;
        call_s += d;
        max_call = std::max(max_call, d);
        return rc;
    };
    auto poll = [&](bool account) -> int {
        for (;;) {
            int64_t k = 0;
            const int rc = timed([&] {
                k = vx_poll(ctx, cq.data(), cq.size());
                return k < 0 ? (int)k : 0;
            }, poll_s);
            if (rc) return rc;
            const auto now = clk::now();
            for (int64_t j = 0; j < k; ++j) {
                const uint32_t b = (uint32_t)cq[j].tag;
                if (account) lat.push_back(since(t_sub[b], now));
                wrong += (cq[j].matched != 0) != (b % 97 != 0);
                free_bufs.push_back(b);
            }
            polled += (uint64_t)k;
            if ((size_t)k < cq.size()) return 0;
        }
    };
    vx_reset_stats(ctx);
    const auto t0 = clk::now();
    auto last = t0;
    double owed = 0;  // bytes arrived but not yet submitted
    for (auto next = t0; since(t0, clk::now()) < seconds; next += std::chrono::microseconds((int64_t)(tick * 1e6))) {
        std::this_thread::sleep_until(next);
        const auto now = clk::now();
        if (since(next, now) > tick) ++late_turns;  // the loop fell behind its cadence
        owed += rate * since(last, now);
        last = now;
        ++turns;
        while (owed >= plen) {
            if (free_bufs.empty()) {
                ++pool_waits;  // every buffer is being hashed: this piece waits for the next turn
                break;
            }
            const uint32_t b = free_bufs.back();
            free_bufs.pop_back();
            t_sub[b] = clk::now();
            if (int rc = timed([&] { return vx_submit(ctx, b, ptrs[b], plen, &digests[(size_t)b * 20]); }, submit_s)) {
                std::fprintf(stderr, "vx_submit: %d %s\n", rc, vx_last_error());
                return 1;
            }
            ++submitted;
            owed -= plen;
        }
        if (timed([&] { return vx_flush(ctx); }, flush_s) || poll(true)) return 1;
    }
    const double wall = since(t0, clk::now());
    vx_stats st{};
    vx_get_stats(ctx, &st);
    // the tail: pieces still in flight at the end (their latency counts too)
    const auto t_end = clk::now();
    while (polled < submitted) {
        if (vx_flush(ctx) || poll(true)) return 1;
        if (since(t_end, clk::now()) > 30) return 4;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    for (uint32_t b = 0; b < nbuf; ++b) {
        vx_unregister_host_buffer(ctx, bufs[b]);
        munmap(bufs[b], plen);
    }
    vx_destroy(ctx);
    const double gib = (double)(1ull << 30);
    std::printf("{\"piece_len\": %u, \"target_GBps\": %.3f, \"achieved_GBps\": %.3f, \"achieved_GiBps\": %.3f, "
                "\"seconds\": %.3f, \"tick_us\": %.0f, \"turns\": %llu, \"late_turns\": %llu, \"pieces\": %llu, "
                "\"pool_buffers\": %u, \"pool_waits\": %llu, \"mismatched_verdicts\": %llu, "
                "\"loop_ms_per_s\": %.3f, \"submit_ms_per_s\": %.3f, \"flush_ms_per_s\": %.3f, \"poll_ms_per_s\": %.3f, "
                "\"max_call_ms\": %.3f, \"submit_stall_ms_per_s\": %.3f, \"batches\": %llu, "
                "\"latency_ms\": {\"p50\": %.3f, \"p90\": %.3f, \"p99\": %.3f, \"max\": %.3f}}\n",
                plen, rate * 1e-9, submitted * (double)plen / wall * 1e-9, submitted * (double)plen / wall / gib,
                wall, tick * 1e6, (unsigned long long)turns, (unsigned long long)late_turns,
                (unsigned long long)submitted, nbuf, (unsigned long long)pool_waits, (unsigned long long)wrong,
                call_s / wall * 1e3, submit_s / wall * 1e3, flush_s / wall * 1e3, poll_s / wall * 1e3, max_call * 1e3,
                st.submit_stall_ns * 1e-6 / wall, (unsigned long long)st.batches, pct(lat, 0.5) * 1e3,
                pct(lat, 0.9) * 1e3, pct(lat, 0.99) * 1e3, pct(lat, 1.0) * 1e3);
    return wrong == 0 && polled == submitted ? 0 : 3;
}
