// vx_files.hpp — host-side pieces of the bulk re-verify from disk
// (vx_verify_files in vx_engine.hip): the torrent file layout, each piece's
// file segments, and a pool of pread threads.
//
// Replaces State::from_metadata_and_root's
//   metadata.pieces.par_iter().enumerate().map(|(idx, hash)|
//       file_store.check_piece_hash_sync(idx, hash)).collect()
// (bittorrent/src/torrent.rs:716-761) with the same per-piece byte ranges as
// FileStore::check_piece_hash_sync (bittorrent/src/file_store.rs:228-303) and
// the file layout of FileStore::new (file_store.rs:126-160).
//
// Pipeline (vx_engine.hip): the readers pread the next slot's pieces straight
// into that slot's pinned stage while the GPU copies and hashes the slots
// already launched; a piece's segments land back to back at its arena offset.
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

#pragma once
#include "vx_hash.h"

namespace vx_files {

struct FileSpan {
    int64_t start_piece, start_offset, end_piece, end_offset, len;
};

// FileStore::new (file_store.rs:126-160).
inline std::vector<FileSpan> layout(const uint64_t* lens, size_t nfiles, uint32_t piece_length) {
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
inline void segments(const std::vector<FileSpan>& fs, int64_t piece, uint32_t piece_length, std::vector<Seg>& out) {
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

inline bool read_full(int fd, uint8_t* dst, int64_t off, int64_t len) {
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

}  // namespace vx_files

