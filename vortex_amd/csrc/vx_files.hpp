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
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>

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
// The reference filters every file of the torrent for each piece
// (files.iter().filter(start_piece <= idx <= end_piece), file_store.rs:238-241),
// which is O(files) per piece and quadratic over a re-verify of a torrent with
// 10^4-10^5 files.  layout() makes start_piece and end_piece non-decreasing in
// the file index (file f+1 starts where file f ends), so the files the filter
// keeps are one contiguous run: the first file with end_piece >= piece (binary
// search) up to the last with start_piece <= piece.  Same files, same order,
// same segments as the walk (tests/test_native_cpu.py checks 10^5 files).
inline void segments(const std::vector<FileSpan>& fs, int64_t piece, uint32_t piece_length, std::vector<Seg>& out) {
    out.clear();
    int64_t total = 0;
    const size_t f0 = (size_t)(std::lower_bound(fs.begin(), fs.end(), piece,
                                                [](const FileSpan& s, int64_t p) { return s.end_piece < p; }) -
                               fs.begin());
    for (size_t f = f0; f < fs.size(); ++f) {
        const FileSpan& s = fs[f];
        if (s.start_piece > piece) break;  // and so does every later file
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
// the piece's concatenated segments) into dst.  A run item (file >= 0) is
// instead `pieces` consecutive pieces lying wholly inside file `file` from
// byte file_off on, landing back to back at dst (piece length apart): one
// pread for all of them (see Runs).
struct ReadItem {
    uint8_t* dst;
    uint64_t piece;
    uint64_t start;
    uint64_t len;
    int32_t file = -1;
    uint32_t pieces = 1;
    int64_t file_off = 0;
};

// Reads that skip the page cache when the data is not in it (DESIGN.md §6.1,
// round 3).  vortex's re-verify (file_store.rs:271-296) preads through the
// page cache; at startup the torrent's data is usually not cached, and on the
// MI355X box a buffered cold pread ran 5-12 GiB/s where O_DIRECT of the same
// file ran ~20 GiB/s (16 threads, profiles/r03/disk/; tools/disk_qd_probe.py).
// Once per call, each file's residency is sampled (mincore on a PROT_READ
// mapping of the file, which faults nothing in).  A file the page cache holds
// (nearly) whole is read buffered throughout, and one it (nearly) lacks goes
// O_DIRECT for every aligned range, both with no per-read probe: inside the
// engine a mincore per 256 KiB read cost the warm linux-mint re-verify 13 % at
// the median (profiles/r04/readers).  Only a partly cached file is probed per
// read: if the first page of the range is not resident and destination,
// offset and length are 4 KiB aligned, the range goes through the O_DIRECT
// descriptor.  An unaligned tail, a cached range, or a direct read that fails
// goes through the normal descriptor.  (O_DIRECT reads stay coherent with the
// page cache: the kernel writes back dirty pages of the range first.)  Bytes are the file's either way: the O_DIRECT
// descriptor is a reopen of the caller's own descriptor (/proc/self/fd/N),
// checked to be the same inode, so a path renamed or replaced after the
// buffered open can never mix two files' bytes in one piece.
// (Round 3 also tried O_DIRECT whenever aligned, and RWF_NOWAIT reads from the
// page cache first: neither beat the mincore probe; removed in round 4.)
class DirectIo {
  public:
    static constexpr uint64_t kBlock = 4096;  // covers 512 B and 4 KiB logical blocks
    // Files below kMinFile gain nothing (their segments are short and rarely
    // aligned), and at most kMaxFiles files get a second descriptor and a
    // mapping, so a torrent of 10^5 small files cannot run the process out of
    // descriptors or mappings (vm.max_map_count) in the middle of a call.
    static constexpr uint64_t kMinFile = 1ull << 20;
    static constexpr size_t kMaxFiles = 4096;
    static constexpr uint64_t kSamples = 256;  // residency samples per call
    // ... but at least this many per file (all pages of a smaller one): with
    // 2 samples a small file of a large torrent, 80 % cached, looked all
    // cached and was read buffered throughout
    static constexpr uint64_t kMinSamples = 16;
    static constexpr double kWarm = 0.9;       // a file this cached is read buffered throughout
    static constexpr double kCold = 0.1;       // one this uncached goes O_DIRECT where aligned, unprobed
    // enabled = false: every read is buffered (vx_config.direct_io = 0).
    DirectIo(const std::vector<int>& fds, bool enabled)
        : dfd_(fds.size(), -1), map_(fds.size(), nullptr), size_(fds.size(), 0), cold_(fds.size(), 0) {
        if (!enabled) return;
        size_t used = 0;
        for (size_t f = 0; f < fds.size() && used < kMaxFiles; ++f) {
            struct stat st;
            if (fds[f] < 0 || fstat(fds[f], &st) != 0 || !S_ISREG(st.st_mode) || st.st_size < (off_t)kMinFile) continue;
            const std::string self = "/proc/self/fd/" + std::to_string(fds[f]);
            const int d = open(self.c_str(), O_RDONLY | O_DIRECT | O_CLOEXEC);
            if (d < 0) continue;  // the filesystem refuses O_DIRECT: buffered reads only
            struct stat dst;
            if (fstat(d, &dst) != 0 || dst.st_dev != st.st_dev || dst.st_ino != st.st_ino) {
                close(d);
                continue;
            }
            void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fds[f], 0);
            if (m == MAP_FAILED) {
                close(d);
                continue;
            }
            dfd_[f] = d;
            map_[f] = m;
            size_[f] = (uint64_t)st.st_size;
            ++used;
        }
        // Residency, sampled once: about kSamples pages spread over the mapped
        // files by size (mid-points of equal parts, at least kMinSamples per
        // file, so a torrent of kMaxFiles files costs ~64,000 mincore calls,
        // a few ms).
        uint64_t total = 0;
        for (size_t f = 0; f < map_.size(); ++f)
            if (map_[f]) total += size_[f];
        uint64_t hit_all = 0, seen_all = 0;
        for (size_t f = 0; f < map_.size() && total; ++f) {
            if (!map_[f]) continue;
            const uint64_t pages = (size_[f] + kBlock - 1) / kBlock;
            const uint64_t k = std::min<uint64_t>(pages, std::max<uint64_t>(kMinSamples, kSamples * size_[f] / total));
            uint64_t hit = 0;
            for (uint64_t i = 0; i < k; ++i)
                hit += resident((uint32_t)f, (int64_t)(((2 * i + 1) * pages / (2 * k)) * kBlock)) ? 1 : 0;
            hit_all += hit;
            seen_all += k;
            if ((double)hit >= kWarm * (double)k) {  // cached: buffered reads, no probe, no second descriptor
                close(dfd_[f]);
                munmap(map_[f], (size_t)size_[f]);
                dfd_[f] = -1;
                map_[f] = nullptr;
            } else if ((double)hit <= kCold * (double)k) {  // not cached: aligned reads go direct, no probe
                munmap(map_[f], (size_t)size_[f]);
                map_[f] = nullptr;
                cold_[f] = 1;
            }
        }
        resident_ = seen_all ? (double)hit_all / (double)seen_all : 1.0;
    }
    ~DirectIo() {
        for (size_t f = 0; f < dfd_.size(); ++f) {
            if (dfd_[f] >= 0) close(dfd_[f]);
            if (map_[f]) munmap(map_[f], (size_t)size_[f]);
        }
    }
    DirectIo(const DirectIo&) = delete;
    DirectIo& operator=(const DirectIo&) = delete;

    // Read [off, off+len) of file f into dst; buffered_fd is the normal descriptor.
    bool read(uint32_t f, int buffered_fd, uint8_t* dst, int64_t off, int64_t len) const {
        const bool aligned = f < dfd_.size() && dfd_[f] >= 0 && len >= (int64_t)kBlock && off >= 0 &&
                             ((reinterpret_cast<uintptr_t>(dst) | (uint64_t)off) & (kBlock - 1)) == 0 &&
                             (uint64_t)(off + len) <= size_[f];
        if (aligned && (cold_[f] || !resident(f, off))) {
            const int64_t head = len & ~(int64_t)(kBlock - 1);
            if (read_full(dfd_[f], dst, off, head)) {
                direct_bytes_.fetch_add((uint64_t)head, std::memory_order_relaxed);
                return head == len || read_full(buffered_fd, dst + head, off + head, len - head);
            }
        }
        return read_full(buffered_fd, dst, off, len);
    }
    uint64_t direct_bytes() const { return direct_bytes_.load(std::memory_order_relaxed); }

    // The sampled fraction of the eligible files' pages the page cache held
    // when this call began.  1 when no file is eligible (O_DIRECT off, or no
    // file it applies to), so the caller's warm choice stands.
    double resident_fraction() const { return resident_; }

  private:
    bool resident(uint32_t f, int64_t off) const {
        unsigned char v = 0;
        return mincore(static_cast<uint8_t*>(map_[f]) + off, 1, &v) != 0 || (v & 1);  // unknown: stay buffered
    }
    std::vector<int> dfd_;
    std::vector<void*> map_;
    std::vector<uint64_t> size_;
    std::vector<uint8_t> cold_;  // sampled as (nearly) uncached: no per-read probe
    double resident_ = 1.0;
    mutable std::atomic<uint64_t> direct_bytes_{0};
};

// Bytes [start, start+len) of a piece, mapped onto its file segments.
inline bool read_range(const std::vector<FileSpan>& fs, const std::vector<int>& fds, uint32_t piece_length,
                       const ReadItem& it, std::vector<Seg>& segs, const DirectIo* dio = nullptr) {
    segments(fs, (int64_t)it.piece, piece_length, segs);
    int64_t pos = 0, at = 0;
    const int64_t a = (int64_t)it.start, b = (int64_t)(it.start + it.len);
    for (const Seg& s : segs) {
        const int64_t lo = std::max<int64_t>(a, pos), hi = std::min<int64_t>(b, pos + s.len);
        if (lo < hi) {
            const bool ok = dio ? dio->read(s.file, fds[s.file], it.dst + at, s.off + (lo - pos), hi - lo)
                                : read_full(fds[s.file], it.dst + at, s.off + (lo - pos), hi - lo);
            if (!ok) return false;
            at += hi - lo;
        }
        pos += s.len;
    }
    return at == (int64_t)it.len;  // short: the files end before the piece does
}

// Coalesced reads for whole pieces.  A piece that lies wholly inside one
// file has a single segment in check_piece_hash_sync's walk
// (file_store.rs:240-298): (piece - start_piece) * piece_length -
// start_offset bytes into that file, the piece's length long.  Consecutive
// such pieces of one file are therefore contiguous in it, and a slot that
// stages pieces piece_length apart can pread the whole run at once instead of
// piece by piece (with 16 KiB pieces the per-piece preads were the bound).
// Pieces that straddle files, or sit in a file that failed to open, keep the
// per-piece walk; a run whose pread fails or reads short is re-read piece by
// piece, so every verdict is the walk's.
class Runs {
  public:
    Runs(const std::vector<FileSpan>& fs, const std::vector<int>& fds, uint32_t piece_length, uint64_t max_bytes)
        : fs_(fs), fds_(fds), pl_(piece_length), max_(max_bytes) {}
    // Append piece `piece` (len bytes, staged at dst) to `out`, extending the
    // last item when it is a run the piece continues.  Pieces must come in
    // increasing order.
    void add(std::vector<ReadItem>& out, uint8_t* dst, uint64_t piece, uint64_t len) {
        const int64_t a = (int64_t)piece * pl_, b = a + (int64_t)len;
        while (f_ < fs_.size() && a >= file_start(f_) + fs_[f_].len) ++f_;
        const bool inside = f_ < fs_.size() && len > 0 && a >= file_start(f_) && b <= file_start(f_) + fs_[f_].len &&
                            fds_[f_] >= 0;
        if (!inside || max_ == 0) {
            out.push_back(ReadItem{dst, piece, 0, len});
            return;
        }
        const int64_t off = a - file_start(f_);
        if (!out.empty()) {
            ReadItem& r = out.back();
            if (r.file == (int32_t)f_ && r.piece + r.pieces == piece && r.len == (uint64_t)r.pieces * pl_ &&
                r.file_off + (int64_t)r.len == off && r.dst + r.len == dst && r.len + len <= max_) {
                r.len += len;
                r.pieces += 1;
                return;
            }
        }
        ReadItem r{dst, piece, 0, len};
        r.file = (int32_t)f_;
        r.file_off = off;
        out.push_back(r);
    }

  private:
    int64_t file_start(size_t f) const { return fs_[f].start_piece * (int64_t)pl_ + fs_[f].start_offset; }
    const std::vector<FileSpan>& fs_;
    const std::vector<int>& fds_;
    const uint32_t pl_;
    const uint64_t max_;
    size_t f_ = 0;
};

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
            uint8_t* bad, uint64_t first = 0, const DirectIo* dio = nullptr)
        : fs_(fs), fds_(fds), pl_(piece_length), bad_(bad), first_(first), dio_(dio) {
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
        done_ns_.push_back(0);
        if (inline_) {
            g.unlock();
            std::vector<Seg> segs;
            for (const ReadItem& it : items) read_item(it, segs);
            g.lock();
            jobs_[id - base_].left = 0;
            jobs_[id - base_].next = items.size();
            done_ns_[id] = now_ns();
            retire();
            return id;
        }
        if (items.empty()) {
            done_ns_[id] = now_ns();
            retire();
        }
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
    // When job `ticket`'s last item finished (steady-clock ns; 0 while unread).
    uint64_t done_ns(uint64_t ticket) {
        std::lock_guard<std::mutex> g(mu_);
        return ticket < done_ns_.size() ? done_ns_[ticket] : 0;
    }
    // Read accounting (vx_tuning_last_verify): pread time summed over threads,
    // bytes, and the first read's start / the last read's end (steady-clock ns).
    uint64_t busy_ns() const { return busy_ns_.load(std::memory_order_relaxed); }
    uint64_t bytes_read() const { return bytes_.load(std::memory_order_relaxed); }
    uint64_t first_start_ns() const { return first_ns_.load(std::memory_order_relaxed); }
    uint64_t first_end_ns() const { return first_end_ns_.load(std::memory_order_relaxed); }
    uint64_t last_end_ns() const { return last_ns_.load(std::memory_order_relaxed); }
    size_t threads() const { return th_.size(); }
    static uint64_t now_ns() {
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    // A run builder over this pool's files (whole-piece slots).
    Runs runs(uint64_t max_bytes) const { return Runs(fs_, fds_, pl_, max_bytes); }
    // Kept for the whole-piece path: one job at a time.
    void start(const std::vector<ReadItem>& items) { (void)submit(items); }

  private:
    struct Job {
        const std::vector<ReadItem>* items;
        size_t next, left;
    };
    // Chunk rounds of one piece may be read by two workers at once (queued
    // jobs), so the bad flag is stored atomically; the caller reads it after
    // wait(), which orders it through mu_.
    void mark_bad(uint64_t piece) { __atomic_store_n(&bad_[piece - first_], (uint8_t)1, __ATOMIC_RELAXED); }
    // Returns the item's read time in ns.
    uint64_t read_item(const ReadItem& it, std::vector<Seg>& segs) {
        const uint64_t t0 = now_ns();
        uint64_t expect = 0;
        first_ns_.compare_exchange_strong(expect, t0, std::memory_order_relaxed);
        read_item_impl(it, segs);
        const uint64_t t1 = now_ns();
        busy_ns_.fetch_add(t1 - t0, std::memory_order_relaxed);
        bytes_.fetch_add(it.len, std::memory_order_relaxed);
        expect = 0;
        first_end_ns_.compare_exchange_strong(expect, t1, std::memory_order_relaxed);
        uint64_t last = last_ns_.load(std::memory_order_relaxed);
        while (last < t1 && !last_ns_.compare_exchange_weak(last, t1, std::memory_order_relaxed)) {
        }
        return t1 - t0;
    }
    void read_item_impl(const ReadItem& it, std::vector<Seg>& segs) {
        if (it.file >= 0) {
            const bool ok = dio_ ? dio_->read((uint32_t)it.file, fds_[it.file], it.dst, it.file_off, (int64_t)it.len)
                                 : read_full(fds_[it.file], it.dst, it.file_off, (int64_t)it.len);
            if (ok) return;
        }
        if (it.file < 0) {
            if (!read_range(fs_, fds_, pl_, it, segs, dio_)) mark_bad(it.piece);
            return;
        }
        for (uint32_t k = 0; k < it.pieces; ++k) {  // the run failed: piece by piece, as the walk reads
            const uint64_t len = k + 1 < it.pieces ? pl_ : it.len - (uint64_t)k * pl_;
            const ReadItem one{it.dst + (uint64_t)k * pl_, it.piece + k, 0, len};
            if (!read_range(fs_, fds_, pl_, one, segs)) mark_bad(one.piece);
        }
    }
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
            (void)read_item(it, segs);
            g.lock();
            if (--jobs_[id - base_].left == 0) {  // the job cannot have retired: left was > 0
                done_ns_[id] = now_ns();
                retire();
            }
        }
    }

    const std::vector<FileSpan>& fs_;
    const std::vector<int>& fds_;
    const uint32_t pl_;
    uint8_t* bad_;
    const uint64_t first_;
    const DirectIo* dio_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    bool stop_ = false, inline_ = false;
    std::deque<Job> jobs_;
    std::vector<uint64_t> done_ns_;  // per ticket: when its reads finished (the re-verify's round timeline)
    uint64_t base_ = 0;  // id of jobs_.front()
    std::atomic<uint64_t> busy_ns_{0}, bytes_{0}, first_ns_{0}, first_end_ns_{0}, last_ns_{0};
};

}  // namespace vx_files

