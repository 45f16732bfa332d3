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
#include <deque>
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

// A fixed pool of reader threads working through a FIFO of read jobs (one
// job = one round's items).  Workers always take the oldest job's next item,
// so jobs finish roughly in submission order, and a worker never idles while
// any submitted item is unread: the re-verify keeps several rounds queued so
// the reads run back to back however the copies are paced.
// An item that fails or reads short marks bad[piece - first] = 1.  `first`
// is the first piece of the verified range.
class Readers {
  public:
    Readers(int n, const std::vector<FileSpan>& fs, const std::vector<int>& fds, uint32_t piece_length,
            uint8_t* bad, uint64_t first = 0)
        : fs_(fs), fds_(fds), pl_(piece_length), bad_(bad), first_(first) {
        for (int t = 0; t < n; ++t) {
            try {
                th_.emplace_back([this] { loop(); });
            } catch (...) {  // no more threads: the ones already started do the reads
                break;
            }
        }
        if (th_.empty()) inline_ = true;  // not even one: submit() reads on the caller's thread
    }
    ~Readers() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // Queue `items` and return its ticket.  The caller keeps the vector
    // unchanged until wait(ticket) (or wait()) has returned: a worker indexes
    // it only under the lock and only while the job has untaken items.
    uint64_t submit(const std::vector<ReadItem>& items) {
        std::unique_lock<std::mutex> g(mu_);
        const uint64_t id = base_ + jobs_.size();
        jobs_.push_back(Job{&items, 0, items.size()});
        if (inline_) {
            g.unlock();
            std::vector<Seg> segs;
            for (const ReadItem& it : items)
                if (!read_range(fs_, fds_, pl_, it, segs)) bad_[it.piece - first_] = 1;
            g.lock();
            jobs_[id - base_].left = 0;
            jobs_[id - base_].next = items.size();
            retire();
            return id;
        }
        if (items.empty()) retire();
        g.unlock();
        cv_.notify_all();
        return id;
    }
    // Block until job `ticket` is read.
    void wait(uint64_t ticket) {
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return ticket < base_ || jobs_[ticket - base_].left == 0; });
    }
    // Block until every submitted job is read.
    void wait() {
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return jobs_.empty(); });
    }
    void run(const std::vector<ReadItem>& items) { wait(submit(items)); }
    // Kept for the whole-piece path: one job at a time.
    void start(const std::vector<ReadItem>& items) { (void)submit(items); }

  private:
    struct Job {
        const std::vector<ReadItem>* items;
        size_t next, left;
    };
    // Drop finished jobs from the front (mu_ held); ids stay base_ + index.
    void retire() {
        while (!jobs_.empty() && jobs_.front().left == 0) {
            jobs_.pop_front();
            ++base_;
        }
        done_cv_.notify_all();
    }
    // The oldest job with an untaken item (mu_ held), or -1.
    long pick() const {
        for (size_t j = 0; j < jobs_.size(); ++j)
            if (jobs_[j].next < jobs_[j].items->size()) return (long)j;
        return -1;
    }
    void loop() {
        std::vector<Seg> segs;
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            cv_.wait(g, [&] { return stop_ || pick() >= 0; });
            if (stop_) return;
            const uint64_t id = base_ + (uint64_t)pick();
            Job& j = jobs_[id - base_];
            const ReadItem& it = (*j.items)[j.next++];
            g.unlock();
            const bool ok = read_range(fs_, fds_, pl_, it, segs);
            g.lock();
            if (!ok) bad_[it.piece - first_] = 1;
            if (--jobs_[id - base_].left == 0) retire();  // the job cannot have retired: left was > 0
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
    bool stop_ = false, inline_ = false;
    std::deque<Job> jobs_;
    uint64_t base_ = 0;  // id of jobs_.front()
};

}  // namespace vx_files

