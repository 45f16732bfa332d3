// vx_files.cpp — bulk re-verify of a torrent's files on disk, on top of the
// public C ABI (vx_submit / vx_flush / vx_poll).
//
// Replaces State::from_metadata_and_root's
//   metadata.pieces.par_iter().enumerate().map(|(idx, hash)|
//       file_store.check_piece_hash_sync(idx, hash)).collect()
// (bittorrent/src/torrent.rs:716-761) with the same per-piece byte ranges as
// FileStore::check_piece_hash_sync (bittorrent/src/file_store.rs:228-303) and
// the file layout of FileStore::new (file_store.rs:126-160).
//
// Pipeline: io_threads readers pread batch k+1 into pinned (registered) host
// buffers while the GPU hashes batch k; two host batches alternate.  A piece
// is read into one contiguous buffer slot (segments back to back), so the
// engine DMAs whole host batches with one copy per engine slot.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "vx_hash.h"

namespace {

struct FileSpan {
    int64_t start_piece, start_offset, end_piece, end_offset, len;
};

// FileStore::new (file_store.rs:126-160).
std::vector<FileSpan> layout(const uint64_t* lens, size_t nfiles, uint32_t piece_length) {
    std::vector<FileSpan> out;
    int64_t sp = 0, so = 0;
    for (size_t f = 0; f < nfiles; ++f) {
        const int64_t L = (int64_t)lens[f];
        const int64_t num = (L + so) / piece_length;
        const int64_t off = (L + so) % piece_length;
        out.push_back(FileSpan{sp, so, sp + num, off, L});
        sp += num;
        so = off;
    }
    return out;
}

struct Seg {
    uint32_t file;
    int64_t off;
    int64_t len;
};

// FileStore::check_piece_hash_sync's segment walk (file_store.rs:240-298).
void segments(const std::vector<FileSpan>& fs, int64_t piece, uint32_t piece_length, std::vector<Seg>& out) {
    out.clear();
    int64_t total = 0;
    for (size_t f = 0; f < fs.size(); ++f) {
        const FileSpan& s = fs[f];
        if (!(s.start_piece <= piece && piece <= s.end_piece)) continue;
        const int64_t file_index = piece - s.start_piece;
        const int64_t file_offset = file_index * (int64_t)piece_length - s.start_offset;
        const int64_t off = file_offset + total;
        int64_t to_read = piece == s.end_piece ? s.end_offset - total
                                               : std::min<int64_t>((int64_t)piece_length - total, s.len);
        if (to_read <= 0) continue;
        out.push_back(Seg{(uint32_t)f, off, to_read});
        total += to_read;
    }
}

bool read_full(int fd, uint8_t* dst, int64_t off, int64_t len) {
    if (fd < 0 || off < 0) return false;
    int64_t got = 0;
    while (got < len) {
        const ssize_t r = pread(fd, dst + got, (size_t)(len - got), (off_t)(off + got));
        if (r <= 0) return false;  // error or unexpected EOF (file_store.rs:283-292)
        got += r;
    }
    return true;
}

// A fixed pool of reader threads; fill(lo, hi) preads pieces [lo, hi).
class Readers {
  public:
    Readers(int n, const std::vector<FileSpan>& fs, const std::vector<int>& fds, uint32_t piece_length,
            uint64_t n_pieces, uint64_t total_len)
        : fs_(fs), fds_(fds), pl_(piece_length), np_(n_pieces), total_(total_len) {
        for (int t = 0; t < n; ++t) th_.emplace_back([this] { run(); });
    }
    ~Readers() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void start(uint64_t lo, uint64_t hi, uint8_t* buf, uint64_t stride, uint8_t* bad) {
        std::lock_guard<std::mutex> g(mu_);
        lo_ = lo;
        hi_ = hi;
        buf_ = buf;
        stride_ = stride;
        bad_ = bad;
        next_.store(lo);
        left_ = hi - lo;
        ++gen_;
        cv_.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return left_ == 0; });
    }
    uint32_t piece_len(uint64_t i) const {
        const uint64_t last = total_ % pl_ ? total_ % pl_ : pl_;
        return i == np_ - 1 ? (uint32_t)last : pl_;
    }

  private:
    void run() {
        std::vector<Seg> segs;
        uint64_t seen = 0;
        for (;;) {
            uint64_t lo, hi, stride;
            uint8_t *buf, *bad;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                lo = lo_;
                hi = hi_;
                buf = buf_;
                stride = stride_;
                bad = bad_;
            }
            uint64_t mine = 0;
            for (;;) {
                const uint64_t i = next_.fetch_add(1);
                if (i >= hi) break;
                segments(fs_, (int64_t)i, pl_, segs);
                uint8_t* dst = buf + (i - lo) * stride;
                bool ok = true;
                int64_t at = 0;
                for (const Seg& s : segs) {
                    ok = ok && read_full(fds_[s.file], dst + at, s.off, s.len);
                    at += s.len;
                }
                ok = ok && at == (int64_t)piece_len(i);
                bad[i] = ok ? 0 : 1;
                ++mine;
            }
            std::lock_guard<std::mutex> g(mu_);
            left_ -= mine;
            if (left_ == 0) done_cv_.notify_all();
        }
    }

    const std::vector<FileSpan>& fs_;
    const std::vector<int>& fds_;
    const uint32_t pl_;
    const uint64_t np_, total_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    bool stop_ = false;
    uint64_t gen_ = 0, lo_ = 0, hi_ = 0, stride_ = 0, left_ = 0;
    uint8_t *buf_ = nullptr, *bad_ = nullptr;
    std::atomic<uint64_t> next_{0};
};

}  // namespace

extern "C" int64_t vx_verify_files(vx_ctx* ctx, const char* const* paths, const uint64_t* file_lengths,
                                   size_t nfiles, uint32_t piece_length, const uint8_t* expected, size_t n_pieces,
                                   uint8_t* matched_out, uint32_t io_threads) {
    if (!ctx || (nfiles && (!paths || !file_lengths)) || piece_length == 0 || (n_pieces && (!expected || !matched_out)))
        return VX_EINVAL;
    if (vx_pending(ctx)) return VX_EBUSY;
    uint64_t total = 0;
    for (size_t f = 0; f < nfiles; ++f) total += file_lengths[f];
    if (n_pieces != (total + piece_length - 1) / piece_length) return VX_EINVAL;
    if (n_pieces == 0) return 0;

    const std::vector<FileSpan> fs = layout(file_lengths, nfiles, piece_length);
    std::vector<int> fds(nfiles, -1);
    for (size_t f = 0; f < nfiles; ++f) fds[f] = open(paths[f], O_RDONLY | O_CLOEXEC);

    const uint64_t stride = (piece_length + 255u) / 256u * 256u;
    const uint64_t per_batch = std::max<uint64_t>(1, std::min<uint64_t>(n_pieces, (256ull << 20) / stride));
    const size_t bytes = (size_t)(per_batch * stride);
    uint8_t* hb[2] = {nullptr, nullptr};
    int64_t rc = 0;
    for (auto& b : hb) {
        b = static_cast<uint8_t*>(std::aligned_alloc(4096, (bytes + 4095) / 4096 * 4096));
        if (!b) rc = VX_ENOMEM;
    }
    bool reg[2] = {false, false};
    for (int k = 0; k < 2 && !rc; ++k) {
        int r = vx_register_host_buffer(ctx, hb[k], (bytes + 4095) / 4096 * 4096);
        if (r) rc = r;
        reg[k] = r == 0;
    }
    std::vector<uint8_t> bad(n_pieces, 0);
    std::memset(matched_out, 0, n_pieces);
    if (!rc) {
        const int nthreads =
            io_threads ? (int)io_threads : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        Readers rd(nthreads, fs, fds, piece_length, n_pieces, total);
        const uint64_t nbatches = (n_pieces + per_batch - 1) / per_batch;
        std::vector<uint64_t> left(nbatches, 0);
        std::vector<vx_completion> cbuf(1024);
        auto poll = [&]() -> int64_t {
            for (;;) {
                const int64_t k = vx_poll(ctx, cbuf.data(), cbuf.size());
                if (k < 0) return k;
                for (int64_t j = 0; j < k; ++j) {
                    const uint64_t i = cbuf[j].tag;
                    matched_out[i] = (cbuf[j].matched && !bad[i]) ? 1 : 0;
                    --left[i / per_batch];
                }
                if ((size_t)k < cbuf.size()) return 0;
            }
        };
        auto wait_batch = [&](uint64_t b) -> int64_t {
            while (left[b]) {
                int64_t r = poll();
                if (r) return r;
                if (left[b]) std::this_thread::sleep_for(std::chrono::microseconds(50));
            }
            return 0;
        };
        auto range = [&](uint64_t b, uint64_t& lo, uint64_t& hi) {
            lo = b * per_batch;
            hi = std::min<uint64_t>(n_pieces, lo + per_batch);
        };
        uint64_t lo, hi;
        range(0, lo, hi);
        rd.start(lo, hi, hb[0], stride, bad.data());
        for (uint64_t b = 0; b < nbatches && !rc; ++b) {
            rd.wait();
            range(b, lo, hi);
            left[b] = hi - lo;
            uint8_t* buf = hb[b & 1];
            for (uint64_t i = lo; i < hi && !rc; ++i) {
                const int r = vx_submit(ctx, i, buf + (i - lo) * stride, rd.piece_len(i), expected + 20 * i);
                if (r) rc = r;
            }
            if (!rc) rc = vx_flush(ctx);
            if (rc) break;
            if (b + 1 < nbatches) {
                // buffer (b+1)&1 was last used by batch b-1: its DMA must be done
                if (b >= 1) rc = wait_batch(b - 1);
                if (rc) break;
                uint64_t lo2, hi2;
                range(b + 1, lo2, hi2);
                rd.start(lo2, hi2, hb[(b + 1) & 1], stride, bad.data());
            }
            rc = poll();
        }
        if (rc) {
            // make sure no reader still writes a buffer we are about to free
            rd.wait();
        }
        if (!rc) rc = vx_drain(ctx, 0);
        if (!rc) rc = poll();
        if (rc) {
            // error path: retire everything still in flight before the
            // buffers are unregistered and freed
            (void)vx_drain(ctx, 0);
            for (int guard = 0; vx_pending(ctx) && guard < 1 << 20; ++guard)
                if (vx_poll(ctx, cbuf.data(), cbuf.size()) <= 0) break;
        }
    }
    for (int k = 0; k < 2; ++k) {
        if (reg[k]) (void)vx_unregister_host_buffer(ctx, hb[k]);
        std::free(hb[k]);
    }
    for (int fd : fds)
        if (fd >= 0) close(fd);
    if (rc) return rc;
    int64_t nbad = 0;
    for (uint8_t x : bad) nbad += x;
    return nbad;
}
