// oracle/pool_oracle.cpp — TEST INFRASTRUCTURE ONLY (CPU restatement of vortex's
// "Parallel hash computations" pool).  Used as the parity checker in tests/ and
// as the timed CPU baseline in bench.py (cpu_baseline.kind = "port"); never
// linked into vortex_amd/.
//
// What it restates (reference is Rust + rayon, not buildable here: no cargo):
//  * Download path: each completed piece is one task on the rayon global pool,
//    `scope.spawn(move |_| { Sha1::new(); update(&buf[..piece_len]); finalize()
//    == metadata.pieces[index]; complete_tx.send(DownloadedPiece{..}) })`
//    — bittorrent/src/peer_comm/peer_connection.rs:1145-1158.
//  * Results travel over std::sync::mpsc (torrent.rs:319-320, 333) and the
//    submitting (event-loop) thread drains them with try_recv
//    (torrent.rs:415-442).
//  * Bulk re-verify is `pieces.par_iter().enumerate().map(check).collect()`
//    (torrent.rs:724-740).
//  * Pool size: rayon's default global pool = one worker per logical CPU; the
//    reference never overrides it (no ThreadPoolBuilder / RAYON_NUM_THREADS).
//    Callers pass the thread count explicitly so the bench can report it.
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

extern "C" {
void vxo_sha1_backend(const uint8_t* data, size_t len, uint8_t out[20], int backend);
void vxo_gen_piece(uint64_t seed, uint64_t piece, uint32_t len, uint32_t corrupt_every, uint8_t* out);
}

namespace {

// DownloadedPiece (piece_selector.rs:311-317) minus the Buffer, which the
// caller keeps: index, hash_matched, plus the digest for bit-exact checks.
struct DownloadedPiece {
    size_t index;
    bool hash_matched;
    uint8_t digest[20];
};

// std::sync::mpsc stand-in: unbounded MPSC queue, many senders, one receiver.
class Mpsc {
  public:
    void send(const DownloadedPiece& p) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(p);
        }
        cv_.notify_one();
    }
    DownloadedPiece recv() {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return !q_.empty(); });
        DownloadedPiece p = q_.front();
        q_.pop_front();
        return p;
    }

  private:
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<DownloadedPiece> q_;
};

template <class Job>
void run_pool(size_t n, int threads, Job job, Mpsc& tx) {
    // Work distribution: a shared task counter (each piece is one task, as
    // with scope.spawn / par_iter; rayon's work stealing degenerates to this
    // for equal-cost independent tasks).
    if (threads < 1) threads = 1;
    std::atomic<size_t> next{0};
    std::vector<std::thread> ws;
    ws.reserve(threads);
    for (int t = 0; t < threads; ++t) {
        ws.emplace_back([&, t] {
            (void)t;
            for (;;) {
                size_t i = next.fetch_add(1, std::memory_order_relaxed);
                if (i >= n) break;
                tx.send(job(i));
            }
        });
    }
    // The submitting thread drains the channel (torrent.rs:415-442).
    for (size_t got = 0; got < n; ++got) (void)got, tx.recv();
    for (auto& w : ws) w.join();
}

}  // namespace

extern "C" {

// Verify n host-resident pieces.  expected: n*20 bytes (nullable → matched
// left untouched); digests_out: n*20 bytes (nullable).  Returns 0.
int vxo_pool_verify(const uint8_t* const* ptrs, const uint32_t* lens, const uint8_t* expected, size_t n,
                    int threads, int backend, uint8_t* matched_out, uint8_t* digests_out) {
    Mpsc ch;
    std::vector<DownloadedPiece> results(n);
    auto job = [&](size_t i) {
        DownloadedPiece p;
        p.index = i;
        vxo_sha1_backend(ptrs[i], lens[i], p.digest, backend);
        p.hash_matched = expected ? std::memcmp(p.digest, expected + 20 * i, 20) == 0 : false;
        results[i] = p;  // disjoint slots; also sent through the channel below
        return p;
    };
    run_pool(n, threads, job, ch);
    for (size_t i = 0; i < n; ++i) {
        if (matched_out) matched_out[i] = results[i].hash_matched ? 1 : 0;
        if (digests_out) std::memcpy(digests_out + 20 * i, results[i].digest, 20);
    }
    return 0;
}

// Same pool over synthetic pieces [first, first+n) generated per task into a
// per-thread buffer, so 16 GiB batches can be checked without holding them in
// host memory.  Piece i has length piece_len, except global index
// last_index (if < UINT64_MAX) which has last_len (piece_selector.rs:291-298).
int vxo_pool_digest_synth(uint64_t seed, uint64_t first, size_t n, uint32_t piece_len, uint64_t last_index,
                          uint32_t last_len, uint32_t corrupt_every, int threads, int backend,
                          uint8_t* digests_out) {
    Mpsc ch;
    if (threads < 1) threads = 1;
    std::vector<std::vector<uint8_t>> bufs(threads);
    std::atomic<int> slot{0};
    thread_local int my_slot = -1;
    thread_local const void* my_owner = nullptr;
    auto job = [&](size_t i) {
        if (my_owner != &bufs) {
            my_slot = slot.fetch_add(1);
            my_owner = &bufs;
        }
        std::vector<uint8_t>& b = bufs[my_slot];
        uint64_t g = first + i;
        uint32_t len = (g == last_index) ? last_len : piece_len;
        if (b.size() < len) b.resize(len);
        vxo_gen_piece(seed, g, len, corrupt_every, b.data());
        DownloadedPiece p;
        p.index = i;
        p.hash_matched = false;
        vxo_sha1_backend(b.data(), len, p.digest, backend);
        std::memcpy(digests_out + 20 * i, p.digest, 20);
        return p;
    };
    run_pool(n, threads, job, ch);
    return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Bulk re-verify from files, restated: State::from_metadata_and_root's
// par_iter over FileStore::check_piece_hash_sync (torrent.rs:724-740,
// file_store.rs:228-303).  Per piece: walk the overlapping files, allocate a
// fresh buffer per segment (file_store.rs:272), pread it fully, feed the
// hasher; any I/O error or short read -> false (torrent.rs:731-737).
// ---------------------------------------------------------------------------
#include <fcntl.h>
#include <unistd.h>

extern "C" {
size_t vxo_sha1_ctx_size(void);
void vxo_sha1_init(void* c, int backend);
void vxo_sha1_update(void* c, const uint8_t* p, size_t n);
void vxo_sha1_final(void* c, uint8_t out[20]);

namespace {
// The pool's claim source: piece indices from a counter over [0, n) (the
// plain par_iter), or from a caller's claim function (the split,
// include/vx_hash.h vx_split_claim / vx_split_done: vortex's rayon threads
// asking the engine's claim word for the next piece).
struct Claims {
    int64_t (*claim)(void*) = nullptr;
    void (*done)(void*, uint64_t) = nullptr;
    void* arg = nullptr;
    uint64_t base = 0;  // matched_out[i - base]
};
int pool_verify_files_impl(const char* const* paths, const uint64_t* lens, size_t nfiles, uint32_t piece_length,
                           const uint8_t* expected, size_t n, int threads, int backend, uint8_t* matched_out,
                           const Claims* cl);
}  // namespace

int vxo_pool_verify_files(const char* const* paths, const uint64_t* lens, size_t nfiles, uint32_t piece_length,
                          const uint8_t* expected, size_t n, int threads, int backend, uint8_t* matched_out) {
    return pool_verify_files_impl(paths, lens, nfiles, piece_length, expected, n, threads, backend, matched_out,
                                  nullptr);
}

// The same check_piece_hash_sync per piece, on `threads` threads that take
// their pieces from claim(arg) until it returns -1, write matched_out[i -
// base] and call done(arg, 1) after each verdict.  Returns the pieces taken.
int64_t vxo_pool_verify_files_claim(const char* const* paths, const uint64_t* lens, size_t nfiles,
                                    uint32_t piece_length, const uint8_t* expected, int threads, int backend,
                                    int64_t (*claim)(void*), void (*done)(void*, uint64_t), void* arg, uint64_t base,
                                    uint8_t* matched_out) {
    if (!claim) return -1;
    Claims cl{claim, done, arg, base};
    return pool_verify_files_impl(paths, lens, nfiles, piece_length, expected, 0, threads, backend, matched_out, &cl);
}
}  // extern "C"

namespace {
int pool_verify_files_impl(const char* const* paths, const uint64_t* lens, size_t nfiles, uint32_t piece_length,
                           const uint8_t* expected, size_t n, int threads, int backend, uint8_t* matched_out,
                           const Claims* cl) {
    struct Span { int64_t sp, so, ep, eo, len; };
    std::vector<Span> fs;
    int64_t sp = 0, so = 0;
    for (size_t f = 0; f < nfiles; ++f) {  // FileStore::new, file_store.rs:126-160
        const int64_t L = (int64_t)lens[f];
        fs.push_back(Span{sp, so, sp + (L + so) / piece_length, (L + so) % piece_length, L});
        sp = fs.back().ep;
        so = fs.back().eo;
    }
    std::vector<int> fds(nfiles);
    for (size_t f = 0; f < nfiles; ++f) fds[f] = open(paths[f], O_RDONLY | O_CLOEXEC);
    std::vector<uint8_t> result(n, 0);
    // backend bit 0x100 (diagnostics only, tools/split_alloc_ab.py): read each
    // segment into one buffer per thread instead of a fresh zeroed Vec per
    // segment (file_store.rs:272), to see what the allocation costs the host
    const bool reuse = (backend & 0x100) != 0;
    const int sha_backend = backend & 0xff;
    auto job = [&](size_t idx) {
        DownloadedPiece p;
        p.index = idx;
        thread_local std::vector<uint8_t> ctx;  // the hasher (sha1::Sha1::new(), on the stack in vortex)
        ctx.resize(vxo_sha1_ctx_size());
        vxo_sha1_init(ctx.data(), sha_backend);
        thread_local std::vector<uint8_t> reused;
        const int64_t piece = (int64_t)idx;
        int64_t total = 0;
        bool ok = true;
        for (size_t f = 0; f < fs.size() && ok; ++f) {
            const Span& s = fs[f];
            if (!(s.sp <= piece && piece <= s.ep)) continue;
            const int64_t off = (piece - s.sp) * (int64_t)piece_length - s.so + total;
            const int64_t to_read =
                piece == s.ep ? s.eo - total : std::min<int64_t>((int64_t)piece_length - total, s.len);
            if (to_read <= 0) continue;
            std::vector<uint8_t> fresh;
            if (reuse) {
                if (reused.size() < (size_t)to_read) reused.resize((size_t)to_read);
            } else {
                fresh.assign((size_t)to_read, 0);  // vec![0u8; to_read]
            }
            uint8_t* buffer = reuse ? reused.data() : fresh.data();
            int64_t got = 0;
            while (got < to_read && ok) {
                const ssize_t r = fds[f] < 0 ? -1 : pread(fds[f], buffer + got, (size_t)(to_read - got), off + got);
                if (r <= 0) ok = false;
                else got += r;
            }
            if (ok) vxo_sha1_update(ctx.data(), buffer, (size_t)to_read);
            total += to_read;
        }
        vxo_sha1_final(ctx.data(), p.digest);
        p.hash_matched = ok && std::memcmp(p.digest, expected + 20 * idx, 20) == 0;
        if (cl)
            matched_out[idx - cl->base] = p.hash_matched ? 1 : 0;  // claimed pieces: written in place
        else
            result[idx] = p.hash_matched ? 1 : 0;
        return p;
    };
    // par_iter().map(..).collect() (torrent.rs:724-740): each verdict goes
    // straight into its slot, no channel; the split's threads take their
    // pieces from the claim word instead of the counter.
    std::atomic<int64_t> count{0};
    std::atomic<size_t> next{0};
    std::vector<std::thread> ws;
    for (int t = 0; t < std::max(1, threads); ++t)
        ws.emplace_back([&] {
            for (;;) {
                int64_t i;
                if (cl) {
                    if ((i = cl->claim(cl->arg)) < 0) break;
                } else {
                    const size_t k = next.fetch_add(1, std::memory_order_relaxed);
                    if (k >= n) break;
                    i = (int64_t)k;
                }
                (void)job((size_t)i);
                if (cl && cl->done) cl->done(cl->arg, 1);
                count.fetch_add(1, std::memory_order_relaxed);
            }
        });
    for (auto& w : ws) w.join();
    const int64_t taken = cl ? count.load() : 0;
    if (!cl) std::memcpy(matched_out, result.data(), n);
    for (int fd : fds)
        if (fd >= 0) close(fd);
    return taken;
}
}  // namespace
