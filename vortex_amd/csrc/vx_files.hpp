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

// One read job: bytes [start, start+len) of piece `piece` (a sub-range of
// the piece's concatenated segments) into dst.
struct ReadItem {
    uint8_t* dst;
    uint64_t piece;
    uint64_t start;
    uint64_t len;
};

// Bytes [start, start+len) of a piece, mapped onto its file segments.
inline bool read_range(const std::vector<FileSpan>& fs, const std::vector<int>& fds, uint32_t piece_length,
                       const ReadItem& it, std::vector<Seg>& segs) {
    segments(fs, (int64_t)it.piece, piece_length, segs);
    int64_t pos = 0, at = 0;
    const int64_t a = (int64_t)it.start, b = (int64_t)(it.start + it.len);
    for (const Seg& s : segs) {
        const int64_t lo = std::max<int64_t>(a, pos), hi = std::min<int64_t>(b, pos + s.len);
        if (lo < hi) {
            if (!read_full(fds[s.file], it.dst + at, s.off + (lo - pos), hi - lo)) return false;
            at += hi - lo;
        }
        pos += s.len;
    }
    return at == (int64_t)it.len;  // short: the files end before the piece does
}

// A fixed pool of reader threads; run(items) preads every item, marking
// bad[piece - first] = 1 on any I/O error or short read, and returns when all
// are done.  `first` is the first piece of the verified range.
class Readers {
  public:
    Readers(int n, const std::vector<FileSpan>& fs, const std::vector<int>& fds, uint32_t piece_length,
            uint8_t* bad, uint64_t first = 0)
        : fs_(fs), fds_(fds), pl_(piece_length), bad_(bad), first_(first) {
        for (int t = 0; t < n; ++t) th_.emplace_back([this] { loop(); });
    }
    ~Readers() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // The caller may rebuild `items` as soon as run() returns, so a worker
    // takes an item only under the lock and only while the generation it woke
    // for is still the current one: main waits in run() until every taken
    // item is done, so the vector is stable while any worker reads it.  (A
    // lock-free counter let a worker that woke late for a finished
    // generation index the vector while the caller was refilling it.)
    void run(const std::vector<ReadItem>& items) {
        start(items);
        wait();
    }
    // start() hands `items` to the workers and returns; the caller must keep
    // the vector unchanged until wait() returns, and wait() before the next
    // start().  (The re-verify enqueues round k while round k+1 reads.)
    void start(const std::vector<ReadItem>& items) {
        if (items.empty()) return;
        {
            std::lock_guard<std::mutex> g(mu_);
            items_ = &items;
            next_ = 0;
            count_ = items.size();
            left_ = items.size();
            ++gen_;
        }
        cv_.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return left_ == 0; });
    }

  private:
    void loop() {
        std::vector<Seg> segs;
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            for (;;) {
                const ReadItem* it;
                {
                    std::lock_guard<std::mutex> g(mu_);
                    if (gen_ != seen || next_ >= count_) break;  // never touches a finished vector
                    it = &(*items_)[next_++];
                }
                if (!read_range(fs_, fds_, pl_, *it, segs)) bad_[it->piece - first_] = 1;
                std::lock_guard<std::mutex> g(mu_);
                if (--left_ == 0) done_cv_.notify_all();
            }
        }
    }

    const std::vector<FileSpan>& fs_;
    const std::vector<int>& fds_;
    const uint32_t pl_;
    uint8_t* bad_;
    const uint64_t first_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    bool stop_ = false;
    uint64_t gen_ = 0, left_ = 0;
    const std::vector<ReadItem>* items_ = nullptr;
    uint64_t next_ = 0, count_ = 0;
};

}  // namespace vx_files

