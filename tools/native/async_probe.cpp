// async_probe.cpp — throughput of the async download path (vx_submit /
// vx_flush / vx_poll) when completed pieces sit in scattered pool buffers.
//
// vortex hands each completed piece's pool buffer to the hasher
// (peer_connection.rs:1145-1158); consecutive pieces come from unrelated
// buffers of the BufferPool (buf_pool.rs:92-133).  This fills a pool of
// `nbuf` buffers once, takes their digests with vx_sha1_batch, then submits
// `total` pieces from a shuffled buffer order as fast as the engine takes
// them, flushing every `flush_every` submits and polling like the event loop
// (event_loop.rs:554-557).  Every completion must match.  Prints one JSON
// line: GiB/s of piece bytes submitted → verdict polled.
//
// usage: async_probe <piece_len> [nbuf=1024] [total_GiB=8] [flush_every=64] [registered=1] [slot_MiB=default (0)] [slots=4]
//                    [overflow_threads=0] [cap=model|measured]
//   registered: 0 = plain memory (staged), 1 = one registered mmap holding all
//   buffers, 2 = one mmap per buffer, each registered (vortex's BufferPool,
//   buf_pool.rs:92-98)
//   overflow_threads > 0: the context refuses instead of blocking
//   (vx_config.refuse_when_full = 1) and every refused piece is hashed by a
//   pool of that many CPU threads (the CPU oracle's SHA-NI SHA-1 standing in
//   for vortex's rayon pool, as INTEGRATION.md's call site hands it the
//   piece); the line then also gives each side's share.  The loop gives a
//   refused piece to the pool only while the pool's backlog is under one GPU
//   batch latency of work (vx_plan_verify's piece_latency_s over
//   cpu_piece_latency_s, times the pool's threads); otherwise it polls and
//   offers the piece to the engine again (both sides full).
//   [cap=model|measured]: "measured" sets that bound from this run instead:
//   the engine's mean batch latency over the warm-up (vx_get_stats) over one
//   piece's SHA-1 time on this host, times the pool's threads.
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#include "vx_hash.h"

extern "C" void vxo_sha1_backend(const uint8_t* data, size_t len, uint8_t out[20], int backend);  // oracle/

// The overflow pool: refused pieces, hashed and compared on `n` threads.
struct Overflow {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<uint32_t> q;
    bool stop = false;
    std::atomic<uint64_t> done{0}, bad{0};
    std::vector<std::thread> th;
    void start(int n, const std::vector<const uint8_t*>& ptrs, uint32_t plen, const std::vector<uint8_t>& dig) {
        for (int t = 0; t < n; ++t)
            th.emplace_back([&, plen] {
                uint8_t d[20];
                for (;;) {
                    uint32_t b;
                    {
                        std::unique_lock<std::mutex> g(mu);
                        cv.wait(g, [&] { return stop || !q.empty(); });
                        if (q.empty()) return;
                        b = q.front();
                        q.pop_front();
                    }
                    vxo_sha1_backend(ptrs[b], plen, d, 0);
                    if (std::memcmp(d, &dig[(size_t)b * 20], 20) != 0) bad++;
                    done++;
                }
            });
    }
    size_t waiting() {
        std::lock_guard<std::mutex> g(mu);
        return q.size();
    }
    void push(uint32_t b) {
        {
            std::lock_guard<std::mutex> g(mu);
            q.push_back(b);
        }
        cv.notify_one();
    }
    void finish() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
    }
};

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s piece_len [nbuf] [total_GiB] [flush_every] [registered]\n", argv[0]);
        return 2;
    }
    const uint32_t plen = (uint32_t)std::strtoul(argv[1], nullptr, 0);
    const uint32_t nbuf = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 1024;
    const double total_gib = argc > 3 ? std::atof(argv[3]) : 8.0;
    const uint32_t flush_every = argc > 4 ? (uint32_t)std::atoi(argv[4]) : 64;
    const int registered = argc > 5 ? std::atoi(argv[5]) : 1;
    const uint64_t total = (uint64_t)(total_gib * (1ull << 30) / plen);

    vx_config cfg;
    vx_config_default(&cfg, plen);
    if (argc > 6 && std::strtoull(argv[6], nullptr, 0) > 0) {
        cfg.slot_bytes = std::strtoull(argv[6], nullptr, 0) << 20;
        cfg.batch_pieces = (uint32_t)std::min<uint64_t>(65536, cfg.slot_bytes / ((plen + 255) / 256 * 256));
    }
    if (argc > 7) cfg.slots = (uint32_t)std::atoi(argv[7]);  // batch slots (default 4)
    const int overflow_threads = argc > 8 ? std::atoi(argv[8]) : 0;
    const bool cap_measured = argc > 9 && std::strcmp(argv[9], "measured") == 0;
    cfg.refuse_when_full = overflow_threads > 0 ? 1 : 0;
    vx_ctx* ctx = nullptr;
    if (int rc = vx_create(&cfg, &ctx)) {
        std::fprintf(stderr, "vx_create: %d %s\n", rc, vx_last_error());
        return 1;
    }
    const size_t pool_bytes = (size_t)nbuf * plen;
    std::vector<uint8_t*> maps;  // what to unregister / unmap
    auto map = [&](size_t bytes) -> uint8_t* {
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
        return m == MAP_FAILED ? nullptr : static_cast<uint8_t*>(m);
    };
    std::vector<const uint8_t*> ptrs(nbuf);
    std::vector<uint32_t> lens(nbuf, plen);
    if (registered == 2) {
        for (uint32_t b = 0; b < nbuf; ++b) {
            uint8_t* m = map(plen);
            if (!m) return 1;
            maps.push_back(m);
            ptrs[b] = m;
        }
    } else {
        uint8_t* pool = map(pool_bytes);
        if (!pool) return 1;
        maps.push_back(pool);
        for (uint32_t b = 0; b < nbuf; ++b) ptrs[b] = pool + (size_t)b * plen;
    }
    std::mt19937_64 rng(plen);
    for (uint32_t b = 0; b < nbuf; ++b)
        for (size_t i = 0; i < plen / 8; ++i) reinterpret_cast<uint64_t*>(const_cast<uint8_t*>(ptrs[b]))[i] = rng();
    const size_t map_bytes = registered == 2 ? plen : pool_bytes;
    if (registered) {
        for (uint8_t* m : maps)
            if (int rc = vx_register_host_buffer(ctx, m, map_bytes)) {
                std::fprintf(stderr, "register: %d %s\n", rc, vx_last_error());
                return 1;
            }
    }
    std::vector<uint8_t> digests((size_t)nbuf * 20);
    if (int rc = vx_sha1_batch(ctx, ptrs.data(), lens.data(), nbuf, digests.data())) {
        std::fprintf(stderr, "vx_sha1_batch: %d %s\n", rc, vx_last_error());
        return 1;
    }
    std::vector<uint32_t> order(nbuf);
    std::iota(order.begin(), order.end(), 0);
    std::vector<vx_completion> cq(4096);
    uint64_t polled = 0, bad = 0;
    auto poll = [&]() -> int {
        for (;;) {
            const int64_t k = vx_poll(ctx, cq.data(), cq.size());
            if (k < 0) return (int)k;
            for (int64_t j = 0; j < k; ++j) bad += cq[j].matched ? 0 : 1;
            polled += (uint64_t)k;
            if ((size_t)k < cq.size()) return 0;
        }
    };
    // warm-up: four passes over the pool with the timed flush cadence, so
    // every slot has run (and allocated its pinned stage, if it needs one)
    vx_reset_stats(ctx);  // the warm-up's batch latency (cap=measured)
    uint64_t sent = 0;
    for (int pass = 0; pass < 4; ++pass) {
        std::shuffle(order.begin(), order.end(), rng);
        for (uint32_t b : order) {
            int rc;
            while ((rc = vx_submit(ctx, b, ptrs[b], plen, &digests[(size_t)b * 20])) == VX_EBUSY)
                if (poll()) return 1;  // refuse_when_full: the warm-up waits for the GPU itself
            if (rc) {
                std::fprintf(stderr, "warm-up vx_submit: %d %s\n", rc, vx_last_error());
                return 1;
            }
            if (++sent % flush_every == 0 && (vx_flush(ctx) || poll())) return 1;
        }
    }
    if (vx_drain(ctx, 0) || poll()) return 1;
    polled = 0;
    bad = 0;
    sent = 0;
    Overflow ov;
    size_t backlog_cap = 0;
    double gpu_latency_s = 0, cpu_piece_s = 0;
    if (overflow_threads > 0) {
        if (cap_measured) {
            vx_stats ws{};
            vx_get_stats(ctx, &ws);
            gpu_latency_s = ws.batch_latency_count ? ws.batch_latency_sum_us * 1e-6 / ws.batch_latency_count : 0.0;
            uint8_t d[20];
            const int k = 8;
            const double c0 = now_s();
            for (int i = 0; i < k; ++i) vxo_sha1_backend(ptrs[i % nbuf], plen, d, 0);
            cpu_piece_s = (now_s() - c0) / k;
        } else {
            vx_plan pl{};
            vx_plan_verify(1, plen, plen, (uint32_t)overflow_threads, 0.0, &pl);
            gpu_latency_s = pl.piece_latency_s;
            cpu_piece_s = pl.cpu_piece_latency_s;
        }
        ov.start(overflow_threads, ptrs, plen, digests);
        backlog_cap = (size_t)overflow_threads *
                      (size_t)std::max(1.0, std::round(gpu_latency_s / std::max(1e-9, cpu_piece_s)));
    }
    uint64_t refused = 0, to_cpu = 0;
    vx_reset_stats(ctx);  // the engine's own view of the timed region (vx_get_stats)
    const double t0 = now_s();
    while (sent < total) {
        std::shuffle(order.begin(), order.end(), rng);
        for (uint32_t b : order) {
            if (sent == total) break;
            int rc;
            while ((rc = vx_submit(ctx, b, ptrs[b], plen, &digests[(size_t)b * 20])) == VX_EBUSY &&
                   overflow_threads > 0) {
                ++refused;
                if (ov.waiting() < backlog_cap) {  // not taken: the loop's own pool hashes it
                    ov.push(b);
                    rc = 0;
                    ++to_cpu;
                    break;
                }
                if (poll()) return 1;  // both sides full: harvest and offer it to the engine again
            }
            if (rc) {
                std::fprintf(stderr, "vx_submit: %d %s\n", rc, vx_last_error());
                return 1;
            }
            if (++sent % flush_every == 0) {
                if (vx_flush(ctx) || poll()) return 1;
            }
        }
    }
    if (vx_drain(ctx, 0) || poll()) return 1;
    if (overflow_threads > 0) ov.finish();
    const double el = now_s() - t0;
    bad += ov.bad.load();
    vx_stats st{};
    vx_get_stats(ctx, &st);
    // median batch latency from the log2 histogram: the bucket holding the middle batch
    uint64_t acc = 0;
    int med = 0;
    for (int k = 0; k < VX_STATS_HIST; ++k) {
        acc += st.batch_latency_hist[k];
        if (2 * acc >= st.batch_latency_count) {
            med = k;
            break;
        }
    }
    if (registered)
        for (uint8_t* m : maps) vx_unregister_host_buffer(ctx, m);
    vx_destroy(ctx);
    for (uint8_t* m : maps) munmap(m, map_bytes);
    std::printf("{\"piece_len\": %u, \"pieces\": %llu, \"registered\": %d, \"flush_every\": %u, \"GiBps\": %.3f, "
                "\"overflow_threads\": %d, \"backlog_cap\": %zu, \"cap\": \"%s\", \"cap_gpu_latency_ms\": %.3f, "
                "\"cap_cpu_piece_ms\": %.4f, \"refused\": %llu, \"cpu_pieces\": %llu, "
                "\"mismatched\": %llu, \"polled\": %llu, \"engine\": {\"batches\": %llu, \"pieces_completed\": %llu, "
                "\"gather_tiles\": %llu, \"staged_bytes\": %llu, \"submit_stall_ms\": %.3f, "
                "\"batch_latency_mean_ms\": %.3f, \"batch_latency_max_ms\": %.3f, "
                "\"batch_latency_median_bucket_ms\": [%.3f, %.3f]}}\n",
                plen, (unsigned long long)total, registered, flush_every,
                (double)total * plen / el / (1 << 30), overflow_threads, backlog_cap,
                cap_measured ? "measured" : "model", gpu_latency_s * 1e3, cpu_piece_s * 1e3, (unsigned long long)refused,
                (unsigned long long)ov.done.load(), (unsigned long long)bad, (unsigned long long)polled,
                (unsigned long long)st.batches, (unsigned long long)st.pieces_completed,
                (unsigned long long)st.gather_tiles, (unsigned long long)st.staged_bytes, st.submit_stall_ns * 1e-6,
                st.batch_latency_count ? st.batch_latency_sum_us * 1e-3 / st.batch_latency_count : 0.0,
                st.batch_latency_max_us * 1e-3, (double)(med ? 1ull << med : 0) * 1e-3, (double)(2ull << med) * 1e-3);
    return bad == 0 && polled + ov.done.load() == total ? 0 : 3;
}
