// loop_harness.cpp — test harness: vortex's download-path control flow driven
// against the C ABI (include/vx_hash.h), without io_uring or sockets.
//
// What it mirrors (reference file:line):
//  * BufferPool of 256 piece_length buffers, each its OWN anonymous
//    MAP_POPULATE mmap as in vortex (torrent.rs:344, buf_pool.rs:92-98,
//    buf_ring.rs:24-42), each registered with vx_register_host_buffer so the
//    batch's gather kernel pulls completed pieces straight to the GPU.
//  * Piece::on_subpiece copies each 16 KiB subpiece into the piece buffer
//    (piece_selector.rs:381-398); when the piece is complete it is handed to
//    the hasher (peer_connection.rs:1122-1158) → vx_submit.
//  * Once per loop turn the event loop drains completions
//    (event_loop.rs:554-557 → torrent.rs:415-442) → vx_flush + vx_poll:
//    match → piece complete (buffer returned after the "disk write");
//    mismatch → mark_not_downloaded + return_buffer + re-request.
//  * Buffers are reused without zeroing (buf_pool.rs:148-157); the engine
//    must hash exactly piece_len bytes.
// "Peers" deliver subpieces of synthetic data (DESIGN.md "Synthetic pieces");
// a configurable fraction of first deliveries is corrupted, so the mismatch
// branch runs and the piece is downloaded again.
//
// Faults (INTEGRATION.md "One ownership rule for submits" / "Device
// failure"): with fail_submit_every = K > 0 every K-th submit is refused
// (vx_tuning_fail_submit_after, non-sticky VX_ENOMEM), and with
// fail_launch_after = L >= 0 the (L+1)-th batch launch fails like a device
// error.  The harness then does what INTEGRATION.md's Rust call sites do: a
// refused piece goes to "vortex's own pool" (a small thread pool running the
// CPU restatement of the sha1 closure, oracle/liboracle.so, with results over
// a channel drained each turn); after the device fails, vx_poll is drained
// until it errors, vx_destroy waits for the device, every still-inflight piece
// goes to the CPU pool, and every later piece is hashed there.  Every delivery
// must produce exactly one verdict.
//
// usage: loop_harness <expected.bin> <n_pieces> <piece_len> <last_len> <seed>
//                     [peers=32] [subpieces_per_turn=4] [corrupt_every=50]
//                     [fail_submit_every=0] [fail_launch_after=-1]
// prints one JSON line; exit status 0 iff every piece completed with the
// expected digest and every corrupted delivery was rejected.
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "vx_hash.h"
#include "vx_tuning.h"

extern "C" void vxo_sha1(const uint8_t* data, size_t len, uint8_t out[20]);  // oracle/liboracle.so

namespace {

uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// Synthetic piece bytes [off, off+len) of piece p.
void gen_range(uint64_t seed, uint64_t p, uint32_t off, uint32_t len, uint8_t* out) {
    const uint64_t key = mix64(seed ^ (p * 0xD1B54A32D192ED03ULL));
    for (uint32_t i = 0; i < len;) {
        const uint32_t b = off + i;
        const uint64_t w = mix64(key + (uint64_t)(b / 8 + 1) * 0x9E3779B97F4A7C15ULL);
        const uint32_t k = b % 8;
        const uint32_t take = std::min<uint32_t>(8 - k, len - i);
        std::memcpy(out + i, reinterpret_cast<const uint8_t*>(&w) + k, take);
        i += take;
    }
}

constexpr uint32_t kSubpiece = 16384;  // SUBPIECE_SIZE, piece_selector.rs:15

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// vortex's own pool for pieces the GPU does not take: the reference's closure
// (peer_connection.rs:1145-1158) on worker threads, results over a channel
// (the downloaded_piece_tx/rc pair, torrent.rs:319-320) drained by the loop.
class CpuPool {
  public:
    struct Done {
        uint64_t tag;
        bool matched;
    };
    explicit CpuPool(int threads) {
        for (int t = 0; t < threads; ++t) th_.emplace_back([this] { run(); });
    }
    ~CpuPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void spawn(uint64_t tag, const uint8_t* buf, uint32_t len, const uint8_t* expected) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(Job{tag, buf, len, expected});
        }
        cv_.notify_one();
    }
    void try_recv(std::vector<Done>& out) {
        std::lock_guard<std::mutex> g(mu_);
        out.insert(out.end(), done_.begin(), done_.end());
        done_.clear();
    }
    bool idle() {
        std::lock_guard<std::mutex> g(mu_);
        return q_.empty() && busy_ == 0;
    }

  private:
    struct Job {
        uint64_t tag;
        const uint8_t* buf;
        uint32_t len;
        const uint8_t* expected;
    };
    void run() {
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            cv_.wait(g, [&] { return stop_ || !q_.empty(); });
            if (q_.empty()) return;
            const Job j = q_.front();
            q_.pop_front();
            ++busy_;
            g.unlock();
            uint8_t d[20];
            vxo_sha1(j.buf, j.len, d);
            const bool m = std::memcmp(d, j.expected, 20) == 0;
            g.lock();
            --busy_;
            done_.push_back(Done{j.tag, m});
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Job> q_;
    std::vector<Done> done_;
    int busy_ = 0;
    bool stop_ = false;
};

}  // namespace

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s expected.bin n piece_len last_len seed [peers] [subs/turn] [corrupt_every]\n",
                     argv[0]);
        return 2;
    }
    const char* exp_path = argv[1];
    const uint32_t n = (uint32_t)std::strtoul(argv[2], nullptr, 10);
    const uint32_t plen = (uint32_t)std::strtoul(argv[3], nullptr, 10);
    const uint32_t last_len = (uint32_t)std::strtoul(argv[4], nullptr, 10);
    const uint64_t seed = std::strtoull(argv[5], nullptr, 0);
    const uint32_t peers = argc > 6 ? (uint32_t)std::atoi(argv[6]) : 32;
    const uint32_t subs_per_turn = argc > 7 ? (uint32_t)std::atoi(argv[7]) : 4;
    const uint32_t corrupt_every = argc > 8 ? (uint32_t)std::atoi(argv[8]) : 50;
    const uint32_t fail_submit_every = argc > 9 ? (uint32_t)std::atoi(argv[9]) : 0;
    const int64_t fail_launch_after = argc > 10 ? std::atoll(argv[10]) : -1;

    std::vector<uint8_t> expected((size_t)n * 20);
    FILE* f = std::fopen(exp_path, "rb");
    if (!f || std::fread(expected.data(), 1, expected.size(), f) != expected.size()) {
        std::fprintf(stderr, "cannot read %s\n", exp_path);
        return 2;
    }
    std::fclose(f);

    vx_config cfg;
    vx_config_default(&cfg, plen);
    cfg.slots = 4;
    vx_ctx* ctx = nullptr;
    if (int rc = vx_create(&cfg, &ctx)) {
        std::fprintf(stderr, "vx_create: %d %s\n", rc, vx_last_error());
        return 1;
    }
    // BufferPool: 256 buffers of piece_length (torrent.rs:344), one mmap each.
    const uint32_t nbuf = 256;
    std::vector<uint8_t*> pool(nbuf);
    for (uint32_t b = 0; b < nbuf; ++b) {
        void* m = mmap(nullptr, plen, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
        if (m == MAP_FAILED) return 1;
        pool[b] = static_cast<uint8_t*>(m);
        std::memset(pool[b], 0xEE, plen);  // stale bytes: never zeroed between uses
        if (int rc = vx_register_host_buffer(ctx, pool[b], plen)) {
            std::fprintf(stderr, "register: %d %s\n", rc, vx_last_error());
            return 1;
        }
    }
    std::vector<uint32_t> free_bufs;
    for (uint32_t b = 0; b < nbuf; ++b) free_bufs.push_back(nbuf - 1 - b);
    if (fail_launch_after >= 0) vx_tuning_fail_launch_after(ctx, fail_launch_after);
    CpuPool cpu(4);
    std::unordered_set<uint64_t> on_cpu;  // tags handed to the CPU pool
    bool gpu_dead = false;
    uint64_t refused = 0, cpu_hashed = 0, recovered = 0, submits = 0;

    struct Download {
        uint32_t piece, buf, next_sub, nsub, len;
        bool corrupt;
    };
    std::deque<uint32_t> todo;
    for (uint32_t i = 0; i < n; ++i) todo.push_back(i);
    std::vector<Download> active;
    std::vector<uint8_t> attempts(n, 0), complete(n, 0);
    std::unordered_map<uint64_t, std::pair<uint32_t, double>> inflight;  // tag -> (buf, submit time)
    std::vector<double> lat;
    uint64_t tag_seq = 0, hashed = 0, rejected = 0, wrong = 0, turns = 0, bytes = 0;
    std::vector<vx_completion> cq(512);
    const double t0 = now_ms();
    uint32_t done_count = 0;
    while (done_count < n) {
        ++turns;
        // peers pick pieces (piece picker stand-in: next in order)
        while (active.size() < peers && !todo.empty() && !free_bufs.empty()) {
            const uint32_t p = todo.front();
            todo.pop_front();
            const uint32_t len = p == n - 1 ? last_len : plen;
            const bool corrupt = corrupt_every && attempts[p] == 0 && p % corrupt_every == corrupt_every / 2;
            active.push_back(Download{p, free_bufs.back(), 0, (len + kSubpiece - 1) / kSubpiece, len, corrupt});
            free_bufs.pop_back();
            attempts[p]++;
        }
        // receive: each active download gets subpieces (Piece::on_subpiece)
        for (size_t a = 0; a < active.size();) {
            Download& d = active[a];
            for (uint32_t k = 0; k < subs_per_turn && d.next_sub < d.nsub; ++k, ++d.next_sub) {
                const uint32_t off = d.next_sub * kSubpiece;
                const uint32_t sl = std::min(kSubpiece, d.len - off);
                uint8_t* dst = pool[d.buf] + off;
                gen_range(seed, d.piece, off, sl, dst);
                if (d.corrupt && d.next_sub == d.nsub / 2) dst[sl / 3] ^= 0x40;
            }
            if (d.next_sub == d.nsub) {  // complete → hash (peer_connection.rs:1145)
                const uint64_t tag = (tag_seq++ << 32) | d.piece;
                const uint8_t* buf = pool[d.buf];
                const uint8_t* want = &expected[(size_t)d.piece * 20];
                int rc = VX_EDEVICE;
                if (!gpu_dead) {
                    if (fail_submit_every && ++submits % fail_submit_every == 0) vx_tuning_fail_submit_after(ctx, 0);
                    rc = vx_submit(ctx, tag, buf, d.len, want);
                }
                if (rc != 0) {
                    // not taken (vx_hash.h ownership rule): the reference's closure runs on the CPU pool
                    if (rc != VX_ENOMEM && rc != VX_EDEVICE) {
                        std::fprintf(stderr, "vx_submit: %d %s\n", rc, vx_last_error());
                        return 1;
                    }
                    if (!gpu_dead) ++refused;
                    if (rc == VX_EDEVICE) gpu_dead = true;
                    cpu.spawn(tag, buf, d.len, want);
                    on_cpu.insert(tag);
                    ++cpu_hashed;
                }
                inflight[tag] = {d.buf, now_ms()};
                bytes += d.len;
                active[a] = active.back();
                active.pop_back();
            } else {
                ++a;
            }
        }
        // end of loop turn: drain completions (event_loop.rs:554-557)
        auto verdict = [&](uint64_t tag, bool matched) -> bool {
            const uint32_t p = (uint32_t)(tag & 0xFFFFFFFFu);
            auto it = inflight.find(tag);
            if (it == inflight.end()) return false;  // unknown or duplicate: exactly-once broken
            lat.push_back(now_ms() - it->second.second);
            free_bufs.push_back(it->second.first);  // return_buffer
            inflight.erase(it);
            ++hashed;
            const bool was_corrupt = corrupt_every && attempts[p] == 1 && p % corrupt_every == corrupt_every / 2;
            if (matched) {
                if (was_corrupt) ++wrong;  // corrupted data must never verify
                complete[p] = 1;
                ++done_count;
            } else {
                if (!was_corrupt) ++wrong;  // clean data must always verify
                ++rejected;
                todo.push_back(p);  // mark_not_downloaded → re-request
            }
            return true;
        };
        bool failed_now = false;
        if (ctx) {
            if (vx_flush(ctx) != 0) failed_now = true;
            for (;;) {
                const int64_t k = vx_poll(ctx, cq.data(), cq.size());
                if (k < 0) {
                    failed_now = true;
                    break;
                }
                for (int64_t j = 0; j < k; ++j)
                    if (!verdict(cq[j].tag, cq[j].matched != 0)) return 4;
                if ((size_t)k < cq.size()) break;
            }
        }
        if (failed_now) {
            // device failure: vx_poll has handed out every
            // finished result; vx_destroy waits for the device, then every
            // piece still with the GPU is hashed on the CPU pool.
            for (;;) {  // drain what is left after a flush-time error
                const int64_t k = vx_poll(ctx, cq.data(), cq.size());
                if (k <= 0) break;
                for (int64_t j = 0; j < k; ++j)
                    if (!verdict(cq[j].tag, cq[j].matched != 0)) return 4;
            }
            const uint64_t pending = vx_pending(ctx);
            vx_destroy(ctx);  // waits for the device, unregisters the pool buffers
            ctx = nullptr;
            gpu_dead = true;
            // the GPU's unfinished pieces (take_unfinished): every inflight tag not already on the CPU pool
            uint64_t handed = 0;
            for (const auto& kv : inflight) {
                const uint64_t t = kv.first;
                if (on_cpu.count(t)) continue;
                const uint32_t p = (uint32_t)(t & 0xFFFFFFFFu);
                cpu.spawn(t, pool[kv.second.first], p == n - 1 ? last_len : plen, &expected[(size_t)p * 20]);
                on_cpu.insert(t);
                ++handed;
            }
            recovered += handed;
            if (handed != pending) {
                std::fprintf(stderr, "unfinished %llu != vx_pending %llu\n", (unsigned long long)handed,
                             (unsigned long long)pending);
                return 5;
            }
        }
        std::vector<CpuPool::Done> cdone;
        cpu.try_recv(cdone);
        for (const auto& d : cdone)
            if (!verdict(d.tag, d.matched)) return 4;
        if (active.empty() && todo.empty() && !inflight.empty()) {
            // nothing left to receive: block for the GPU like the loop's
            // CQE wait would (torrent.rs:42, event_loop.rs:438-439)
            if (ctx) vx_drain(ctx, 0);
            else std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    }
    const double el = now_ms() - t0;
    vx_stats st{};  // what the event loop would export under vortex's `metrics` feature
    if (ctx) {
        vx_get_stats(ctx, &st);
        for (uint8_t* b : pool) vx_unregister_host_buffer(ctx, b);
        vx_destroy(ctx);
    }
    for (uint8_t* b : pool) munmap(b, plen);
    std::sort(lat.begin(), lat.end());
    auto pct = [&](double q) { return lat.empty() ? 0.0 : lat[std::min(lat.size() - 1, (size_t)(q * lat.size()))]; };
    std::printf(
        "{\"pieces\": %u, \"piece_len\": %u, \"hashed\": %llu, \"rejected\": %llu, \"wrong\": %llu, \"turns\": %llu, "
        "\"elapsed_ms\": %.1f, \"GiBps\": %.3f, \"latency_ms_p50\": %.2f, \"latency_ms_p99\": %.2f, "
        "\"latency_ms_max\": %.2f, \"engine\": {\"pieces_completed\": %llu, \"pieces_mismatched\": %llu, "
        "\"bytes_completed\": %llu, \"batches\": %llu, \"submit_stall_ms\": %.3f, \"batch_latency_max_ms\": %.3f}, "
        "\"faults\": {\"refused\": %llu, \"cpu_hashed\": %llu, \"recovered\": %llu, \"gpu_dead\": %d}}\n",
        n, plen, (unsigned long long)hashed, (unsigned long long)rejected, (unsigned long long)wrong,
        (unsigned long long)turns, el, bytes / (el * 1e-3) / (1 << 30), pct(0.5), pct(0.99), lat.empty() ? 0 : lat.back(),
        (unsigned long long)st.pieces_completed, (unsigned long long)st.pieces_mismatched,
        (unsigned long long)st.bytes_completed, (unsigned long long)st.batches, st.submit_stall_ns * 1e-6,
        st.batch_latency_max_us * 1e-3, (unsigned long long)refused, (unsigned long long)(cpu_hashed + recovered),
        (unsigned long long)recovered, gpu_dead ? 1 : 0);
    return wrong == 0 && done_count == n ? 0 : 3;
}
