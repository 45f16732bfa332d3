// vx_engine.hip — host side of the C ABI in include/vx_hash.h.
//
// Replaces, on the host, what vortex does around its hashing pool:
//  * vx_submit / vx_flush / vx_poll: the scope.spawn → mpsc → try_recv cycle
//    (peer_connection.rs:1145-1158 → torrent.rs:415-442), batched for the GPU.
//  * vx_sha1_batch / vx_verify_batch: the par_iter bulk verify
//    (torrent.rs:724-740).
//  * vx_sha1_device_*: enqueue the kernels on device-resident batches.
//
// Design (DESIGN.md "Host engine"): a context owns `slots` batch slots, each
// with its own HIP stream, a device arena, a pinned staging arena and pinned
// metadata.  Pieces are appended to the filling slot at 256-byte aligned
// offsets: pieces inside a registered (pinned) host range are pulled at launch
// by one gather kernel through the range's device mapping (vx_gather.hip);
// others go through the slot's pinned stage and move with one H2D per
// contiguous run at launch.  On the async path (vx_submit) the stage copy is
// a memcpy at submit; inside a host batch (vx_*_batch) the copies are
// deferred to launch and split over up to 16 short-lived threads
// (stage_copies), and the call waits for every slot before it returns.
// A launch is H2D(meta) → kernel → D2H(digests, verdicts) → event; slots on
// different streams overlap copy and compute.  vx_poll harvests finished
// slots without blocking.  The async path has no internal threads: like the
// reference's loop, it is driven from the caller's thread.  The file
// re-verify runs a pread reader pool (vx_files.hpp) for the call's duration.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <unordered_map>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "vx_files.hpp"
#include "vx_hash.h"
#include "vx_kernels.h"
#include "vx_synth.h"
#include "vx_tuning.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return VX_EDEVICE;
}

#define VX_HIP(call)                                      \
    do {                                                  \
        hipError_t _e = (call);                           \
        if (_e != hipSuccess) return hip_fail(_e, #call); \
    } while (0)

constexpr uint64_t kAlign = 256;
// zc_loader_wins: the slot size below which a batch is latency-bound
constexpr uint32_t kZcMinPieces = 128;

uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

struct Run {
    uint64_t lo, hi;  // staged byte range [lo, hi) of the arena
};

struct DirectRun {
    const uint8_t* host;  // registered (pinned) source of arena bytes [lo, hi)
    uint64_t lo, hi;
};

struct StageCopy {
    const uint8_t* src;  // unregistered caller bytes for stage [off, off + len)
    uint64_t off;
    uint32_t len;
};

struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    hipEvent_t copied = nullptr;  // this slot's H2D finished on the copy stream
    uint64_t arena_cap = 0;
    uint32_t cap = 0;  // pieces
    uint8_t* d_arena = nullptr;
    uint8_t* h_stage = nullptr;
    uint64_t stage_map = 0;  // > 0: h_stage is a registered mmap of this many bytes (alloc_stage)
    // pinned metadata block: offsets | lens | expected | digests | matched
    uint8_t* h_meta = nullptr;
    uint8_t* d_meta = nullptr;
    uint64_t* h_offsets = nullptr;
    uint32_t* h_lens = nullptr;
    uint8_t* h_expected = nullptr;
    uint8_t* h_digests = nullptr;
    uint8_t* h_matched = nullptr;
    uint32_t* h_pidx = nullptr;  // piece-table rows (vx_submit_piece) / piece ids (chunks)
    uint32_t* d_pidx = nullptr;
    uint64_t* h_poff = nullptr;  // chunked re-verify: chunk offset within its piece
    uint64_t* d_poff = nullptr;
    uint64_t* h_tlen = nullptr;  // chunked re-verify: the piece's total length
    uint64_t* d_tlen = nullptr;
    uint64_t* h_src = nullptr;   // gather: device-mapped source of piece i (0 = not gathered)
    uint64_t* d_src = nullptr;
    uint32_t* h_tfirst = nullptr;  // gather: piece i owns tiles [tfirst[i], tfirst[i+1])
    uint32_t* d_tfirst = nullptr;
    uint32_t gtiles = 0;           // gather tiles of this batch
    uint64_t* d_offsets = nullptr;
    uint32_t* d_lens = nullptr;
    uint8_t* d_expected = nullptr;
    uint8_t* d_digests = nullptr;
    uint8_t* d_matched = nullptr;
    std::vector<uint64_t> tags;
    std::vector<Run> runs;
    std::vector<DirectRun> druns;
    std::vector<StageCopy> staged;  // host batches: stage copies deferred to launch
    uint64_t staged_bytes = 0;
    uint32_t n = 0;
    uint64_t bytes = 0;
    bool uniform = true;
    bool has_expected = false;
    bool use_table = false;  // expected digests come from the device piece table
    bool all_mapped = true;  // every non-empty piece is registered and 16-byte aligned (zero-copy candidate)
    enum State { FREE, FILLING, INFLIGHT } state = FREE;
    uint64_t seq = 0;
    std::chrono::steady_clock::time_point t_open{};  // first piece queued (vx_stats batch latency)
};

}  // namespace

struct vx_ctx {
    // Everything a caller chooses comes in here (vx_config, ABI 2): the
    // engine reads no environment variables.
    vx_config cfg{};
    std::vector<Slot> slots;
    // H2D copies are serialised across slots in launch order, so PCIe moves
    // one batch at a time at full rate and batch k's kernel starts as soon as
    // its own bytes are in, while batch k+1 copies (chain_h2d).  (Copies
    // racing on all slot streams share PCIe and delay every kernel.)
    int last_launched = -1;  // slot whose H2D was enqueued last
    // cfg.verify_cold_chunk, when set, is used for calls whose data is not in
    // the page cache (DirectIo::resident_fraction < 0.5 at the call's start),
    // where the readers go O_DIRECT and the disk binds; warm calls keep
    // verify_chunk_for's choice.  Off by default: 1 MiB cold chunks measured
    // +57 % and +7 % on two boxes but -2 % and -5 % (median of 6 and 10
    // evicted calls) on two more, 512 KiB +4 % (profiles/r03/cold/): the
    // box's disk decides, not the chunk.
    // Per-piece device rows of the chunk paths (state | expected | digest |
    // verdict), kept across calls and grown on demand: allocating them per
    // call cost ~1 ms of a 40 ms e2e batch.
    uint8_t* d_chunk_rows = nullptr;
    uint64_t chunk_rows_cap = 0;
    hipEvent_t chunk_prev = nullptr;
    // Device-resident `pieces` table (vx_set_piece_table).
    uint8_t* d_table = nullptr;
    uint32_t n_table = 0;
    int filling = -1;
    // vx_flush found every other slot in flight and left the filling slot
    // open; vx_poll launches it once a slot frees.
    bool flush_pending = false;
    bool bulk = false;  // inside vx_*_batch: slots fill to capacity, not to batch_pieces
    std::deque<vx_completion> done;
    struct Reg {
        size_t len;
        uint8_t* dev;  // device mapping of the range (hipHostGetDevicePointer)
    };
    std::map<uintptr_t, Reg> registered;
    // The same ranges keyed by start address: vortex submits each piece from
    // the start of its own pool mmap (buf_pool.rs:92-98), so most lookups are
    // one hash probe instead of a tree walk.  16 KiB pieces from 1,024
    // separately registered buffers: 29.7 -> 35.7 GiB/s.
    std::unordered_map<uintptr_t, Reg> registered_at;
    // A slot whose pieces are all registered and aligned is hashed straight
    // out of host memory by the zero-copy kernel, without a gather
    // (sha1_zc_split_kernel), unless cfg.zero_copy is 0.
    // (counted in vx_stats.zero_copy_slots / zero_copy_loader_slots)
    uint64_t pending = 0;
    uint64_t seq = 0;
    int sticky = 0;
#ifdef VX_TEST_HOOKS
    // Fault injection, only in the test build libvortex_amd_tuning.so
    // (vx_tuning_fail_submit_after): the submit after this many more succeeds
    // fails with VX_ENOMEM, the way a failed pinned-stage allocation does;
    // < 0 = off.
    int64_t fail_submit_after = -1;
    // vx_tuning_fail_launch_after: the launch after this many more fails as a
    // device error would, turning the context sticky; < 0 = off.
    int64_t fail_launch_after = -1;
#endif
    vx_stats stats{};  // vx_get_stats (observability counters)
    // harvest() counts mismatches unless the caller overrides verdicts after
    // it (the file re-verify: a piece with an I/O error is counted in
    // io_errors only, FileVerify::consume counts the final verdicts)
    bool harvest_counts_mismatches = true;
    // vx_last_verify: the last file re-verify's time budget, and the timing
    // events around its chunk rounds' data copies (reused across calls)
    vx_verify_trace last_verify{};
    std::vector<hipEvent_t> copy_ev;
    std::vector<vx_verify_round> last_rounds;  // vx_last_verify_rounds
    // the last split call's decisions, one per round formed (vx_tuning_last_split)
    struct SplitDecision {
        double t_ms, pool_rate, engine_rate, block_ns, t_engine_ms, t_pool_ms;
        uint64_t unclaimed, group, lanes, pool_done;
        uint32_t mode, measured;
        double lag_ms;  // the learned lag in t_engine_ms
    };
    std::vector<SplitDecision> last_split;
    // What earlier split calls measured, the next call's cold start: the
    // engine's copy intake
    // (B/s, first copy start to last copy end), the kernel's chain per block,
    // and the pool's bytes/s per thread beside the engine (0 = none yet).
    // Each keeps the last kLearn calls' samples: the next call uses their
    // median (split_learn 1, default), so one call slowed by a host stall
    // does not move the next call's first group — and for the intake their
    // largest: a stall slows the pool as much as the engine's reads, and the
    // pool's side starts from its own rate alone, so the engine's starts from
    // its unstalled one too.  split_learn 0 (test build) uses the running mean
    // instead (each call weighted 1/2).
    struct Learned {
        static constexpr uint32_t kLearn = 5;
        double ring[kLearn] = {}, mean = 0;
        uint32_t n = 0;
        void add(double x) {
            mean = n ? 0.5 * (mean + x) : x;
            ring[n++ % kLearn] = x;
        }
        bool any() const { return n > 0; }
        double top() const { return *std::max_element(ring, ring + std::min(n, kLearn)); }
        double get(int median) const {
            if (!median) return mean;
            double v[kLearn];
            const uint32_t k = std::min(n, kLearn);
            std::copy(ring, ring + k, v);
            std::sort(v, v + k);
            return k % 2 ? v[k / 2] : 0.5 * (v[k / 2 - 1] + v[k / 2]);
        }
    };
    // [0]: calls over page-cached data, [1]: over uncached data (O_DIRECT
    // reads; the disk, not PCIe, feeds the engine): one regime's figures
    // would mislead the other's first group.
    Learned split_rin[2], split_bns[2], split_pool_thread_rate[2];
    int split_learn = 1;
    // How much later the engine's last kernel ended than the first group's
    // T_engine said, less the same for the pool's last verdict and T_pool, in
    // calls where the first group was the engine's only one (the readers'
    // start-up and the kernels trailing the copies, which the round model
    // leaves out), kept the same way; the next first group's T_engine adds
    // it.
    Learned split_lag[2];
    int split_lag_on = 1;  // 0: learned, not applied (vx_tuning_split_rules)
    // The file re-verify's chunk rounds put every H2D on this one stream (high
    // priority: its own hardware queue) and only kernels on the slot streams,
    // so no copy ever sits behind a kernel.  Created on first
    // use.  verify_copy_stream = 0 (test build only) restores the slot-stream
    // copies for A/B.
    hipStream_t copy_stream = nullptr;
    int verify_copy_stream = 1;
    // How pinned stages are allocated (alloc_stage): 1 = 2 MiB-aligned mmap
    // with transparent huge pages, then hipHostRegister; 0 = hipHostMalloc
    // (vx_tuning_stage_huge, test build).  Huge pages: warm re-verify 39.1 ->
    // 45.2 GiB/s (its H2D copies 44-47 -> 49-50.5), cold 10.9 -> 14.2, median
    // of 7-9 alternating calls on one box.
    int stage_huge = 1;
    // The split's rules for pieces of one chunk (vx_tuning_split_rules, test
    // build): one_round 1 lets their groups keep claiming while the rates
    // are cold and skips the tenth rule (0: the multi-round rules; 2: as 1,
    // reading piece by piece instead of in runs);
    // round_cap > 0 caps their rounds' bytes (at no fewer than 1,024 lanes),
    // 0: the slot's stage.
    int split_one_round = 1;
    uint64_t split_round_cap = 64ull << 20;
    hipEvent_t anchor_ev = nullptr;            // maps the rounds' GPU times onto the host clock
    uint64_t verify_t0_ns = 0;                 // the running re-verify call's start (steady clock)
};

namespace {

// Pieces (lanes) a slot's metadata holds: the async batch size, or enough
// chunk lanes to fill the arena with kMinChunk-byte chunks (the chunked paths
// of §6.3/§6.4 put one chunk per lane), whichever is larger.
constexpr uint64_t kMinChunk = 64 * 1024;
uint32_t slot_capacity(const vx_config* cfg) {
    return (uint32_t)std::min<uint64_t>(1u << 20, std::max<uint64_t>(cfg->batch_pieces, cfg->slot_bytes / kMinChunk));
}

int set_device(const vx_ctx* c) {
    VX_HIP(hipSetDevice(c->cfg.device));
    return 0;
}

// True if [p, p+len) lies in one registered range; *dev (optional) gets the
// device-mapped address of p.
bool is_registered(const vx_ctx* c, const void* p, size_t len, const uint8_t** dev = nullptr) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    auto hit = c->registered_at.find(a);
    if (hit != c->registered_at.end() && len <= hit->second.len) {
        if (dev) *dev = hit->second.dev;
        return true;
    }
    auto it = c->registered.upper_bound(a);
    if (it == c->registered.begin()) return false;
    --it;
    if (!(a >= it->first && a + len <= it->first + it->second.len)) return false;
    if (dev) *dev = it->second.dev + (a - it->first);
    return true;
}

// Pinned stage memory.  huge: an anonymous mapping aligned to 2 MiB with
// MADV_HUGEPAGE, faulted in, then registered (hipHostRegister), so the
// readers' O_DIRECT reads and the H2D copies touch 512x fewer page-table and
// IOMMU entries than with hipHostMalloc's 4 KiB pages.
uint8_t* alloc_stage(uint64_t bytes, bool huge, uint64_t* mapped) {
    *mapped = 0;
    if (!huge) {
        uint8_t* p = nullptr;
        return hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess ? p : nullptr;
    }
    constexpr uint64_t kHuge = 2ull << 20;
    const uint64_t len = (bytes + kHuge - 1) / kHuge * kHuge;
    void* raw = mmap(nullptr, len + kHuge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (raw == MAP_FAILED) return nullptr;
    const uintptr_t r = reinterpret_cast<uintptr_t>(raw), a = (r + kHuge - 1) / kHuge * kHuge;
    if (a > r) munmap(raw, a - r);  // trim to the aligned [a, a + len)
    if (r + len + kHuge > a + len) munmap(reinterpret_cast<void*>(a + len), r + len + kHuge - (a + len));
    uint8_t* p = reinterpret_cast<uint8_t*>(a);
    (void)madvise(p, len, MADV_HUGEPAGE);  // a hint: 4 KiB pages where THP is off
    // A client that forks (hooks, helpers) must not turn the pinned pages
    // copy-on-write in the parent: the GPU keeps DMAing to the pinned page
    // while a write after the fork would move the parent to a new one.
    (void)madvise(p, len, MADV_DONTFORK);
    for (uint64_t o = 0; o < len; o += 4096) p[o] = 0;
    if (hipHostRegister(p, len, hipHostRegisterDefault) != hipSuccess) {
        munmap(p, len);
        return nullptr;
    }
    *mapped = len;
    return p;
}

void free_stage(Slot& s) {
    if (!s.h_stage) return;
    if (s.stage_map) {
        (void)hipHostUnregister(s.h_stage);
        munmap(s.h_stage, s.stage_map);
    } else {
        (void)hipHostFree(s.h_stage);
    }
    s.h_stage = nullptr;
    s.stage_map = 0;
}

int free_slot_mem(Slot& s) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.copied) (void)hipEventDestroy(s.copied);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    if (s.d_arena) (void)hipFree(s.d_arena);
    if (s.d_meta) (void)hipFree(s.d_meta);
    free_stage(s);
    if (s.h_meta) (void)hipHostFree(s.h_meta);
    s = Slot{};
    return 0;
}

int alloc_slot(Slot& s, uint64_t arena, uint32_t cap) {
    s.arena_cap = arena;
    s.cap = cap;
    VX_HIP(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    VX_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    VX_HIP(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
    if (hipMalloc(&s.d_arena, arena) != hipSuccess) return fail(VX_ENOMEM, "device arena allocation failed");
    // The pinned stage is allocated on first use (ensure_stage): a caller that
    // registers its buffer pool never stages, and pinning slot_bytes of host
    // memory per slot up front would cost as much as the HBM arena.
    // offsets | chunk offsets | total lens | gather sources | lens | piece rows |
    // gather tile prefix (cap+1) | expected | digests | verdicts
    const size_t meta = (size_t)cap * (8 + 8 + 8 + 8 + 4 + 4 + 4 + 20 + 20 + 1) + 64;
    if (hipHostMalloc(&s.h_meta, meta, hipHostMallocDefault) != hipSuccess)
        return fail(VX_ENOMEM, "pinned metadata allocation failed");
    if (hipMalloc(&s.d_meta, meta) != hipSuccess) return fail(VX_ENOMEM, "device metadata allocation failed");
    auto carve = [cap](uint8_t* b, uint64_t*& off, uint64_t*& poff, uint64_t*& tlen, uint64_t*& src,
                       uint32_t*& lens, uint32_t*& pidx, uint32_t*& tfirst, uint8_t*& exp, uint8_t*& dig,
                       uint8_t*& m) {
        size_t at = 0;
        auto take = [&](size_t bytes) {
            uint8_t* p = b + at;
            at += bytes;
            return p;
        };
        off = reinterpret_cast<uint64_t*>(take((size_t)cap * 8));
        poff = reinterpret_cast<uint64_t*>(take((size_t)cap * 8));
        tlen = reinterpret_cast<uint64_t*>(take((size_t)cap * 8));
        src = reinterpret_cast<uint64_t*>(take((size_t)cap * 8));
        lens = reinterpret_cast<uint32_t*>(take((size_t)cap * 4));
        pidx = reinterpret_cast<uint32_t*>(take((size_t)cap * 4));
        tfirst = reinterpret_cast<uint32_t*>(take((size_t)cap * 4 + 4));
        exp = take((size_t)cap * 20);
        dig = take((size_t)cap * 20);
        m = take(cap);
    };
    carve(s.h_meta, s.h_offsets, s.h_poff, s.h_tlen, s.h_src, s.h_lens, s.h_pidx, s.h_tfirst, s.h_expected,
          s.h_digests, s.h_matched);
    carve(s.d_meta, s.d_offsets, s.d_poff, s.d_tlen, s.d_src, s.d_lens, s.d_pidx, s.d_tfirst, s.d_expected,
          s.d_digests, s.d_matched);
    s.h_tfirst[0] = 0;
    s.tags.reserve(cap);
    return 0;
}

// Pinned stage of slot s (unregistered pieces, file reads), allocated on first use.
int ensure_stage(const vx_ctx* c, Slot& s) {
    if (s.h_stage) return 0;
    s.h_stage = alloc_stage(s.arena_cap, c->stage_huge != 0, &s.stage_map);
    if (!s.h_stage && c->stage_huge) s.h_stage = alloc_stage(s.arena_cap, false, &s.stage_map);  // registration refused
    if (!s.h_stage) return fail(VX_ENOMEM, "pinned stage allocation failed");
    return 0;
}

void reset_fill(Slot& s) {
    s.tags.clear();
    s.runs.clear();
    s.druns.clear();
    s.staged.clear();
    s.staged_bytes = 0;
    s.n = 0;
    s.bytes = 0;
    s.gtiles = 0;
    if (s.h_tfirst) s.h_tfirst[0] = 0;
    s.uniform = true;
    s.has_expected = false;
    s.use_table = false;
    s.all_mapped = true;
}

int launch_slot_impl(vx_ctx* c, int si);

// CPUs this process may run on (the container's or cgroup's share, not the
// machine's: hardware_concurrency reports every CPU of a large host).
unsigned usable_cpus() {
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) {
        const int n = CPU_COUNT(&set);
        if (n > 0) return (unsigned)n;
    }
    return std::max(1u, std::thread::hardware_concurrency());
}

// A host batch's unregistered pieces reach the pinned stage here, split by
// bytes over up to 16 threads: one thread's memcpy (~10-13 GiB/s) bounded
// config 3 from plain memory.  The caller's buffers stay
// valid because vx_*_batch returns only after every slot has completed (or,
// on an error, after every in-flight slot has been waited for: abandon_batch).
// A thread that cannot be created leaves its range to the calling thread, so
// no exception crosses the C ABI.
void stage_copies(Slot& s) {
    if (s.staged.empty()) return;
    const uint64_t per = 16ull << 20;
    static const unsigned hw = usable_cpus();
    const unsigned T = (unsigned)std::min<uint64_t>({16, hw, std::max<uint64_t>(1, s.staged_bytes / per)});
    auto copy = [&s](size_t a, size_t b) {
        for (size_t k = a; k < b; ++k) std::memcpy(s.h_stage + s.staged[k].off, s.staged[k].src, s.staged[k].len);
    };
    if (T <= 1) {
        copy(0, s.staged.size());
    } else {
        // contiguous ranges of roughly staged_bytes / T each
        std::vector<size_t> cut{0};
        uint64_t acc = 0, next = s.staged_bytes / T;
        for (size_t k = 0; k < s.staged.size() && cut.size() < T; ++k) {
            acc += s.staged[k].len;
            if (acc >= next) {
                cut.push_back(k + 1);
                next += s.staged_bytes / T;
            }
        }
        cut.push_back(s.staged.size());
        std::vector<std::thread> th;
        th.reserve(cut.size());
        size_t t = 1;
        try {
            for (; t + 1 < cut.size(); ++t) th.emplace_back(copy, cut[t], cut[t + 1]);
        } catch (...) {  // std::system_error (EAGAIN) or bad_alloc: copy the rest here
        }
        copy(cut[0], cut[1]);
        for (size_t u = t; u + 1 < cut.size(); ++u) copy(cut[u], cut[u + 1]);
        for (auto& x : th) x.join();
    }
    s.staged.clear();
    s.staged_bytes = 0;
}

// Order slot si's H2D after the previously launched slot's (one PCIe stream
// of copies across all slots): the host waits for the previous slot's copy,
// with no cross-stream wait.  That keeps copies back to back with a gap of
// one host wake-up and blocks the host for at most one batch's copy.  The
// alternatives measured worse and were removed in round 4 (EXPERIMENTS.md):
// a stream wait on the previous `copied` event blocked hipMemcpyAsync for
// ~8-9 ms at a time and left PCIe idle (34-46 GiB/s, 38-40 with an extra
// host wait two launches back), one dedicated copy stream 45, this 48.5-48.7
// (8192 x 256 KiB through vx_verify_batch, profiles/r01/h2d_modes/).
int chain_h2d(vx_ctx* c, int si) {
    const int last = c->last_launched;
    if (last >= 0 && last != si) VX_HIP(hipEventSynchronize(c->slots[last].copied));
    return 0;
}

void mark_launched(vx_ctx* c, int si) { c->last_launched = si; }

// Run every command type a batch uses once on every slot stream, in the
// launch pattern of launch_slot_impl (cross-slot copy chain, large and small
// H2D, both default kernels, D2H).  The HIP runtime sets up the hardware
// queues and copy paths behind a stream on first use, and that blocked the
// host for ~8 ms inside hipMemcpyAsync on the first two slots of the first
// batches (profiles/r01/e2e_first_use/); paying it here keeps it off the
// batch path.
int warm_slots(vx_ctx* c) {
    int prev = -1;
    for (int si = 0; si < (int)c->slots.size(); ++si) {
        Slot& s = c->slots[si];
        hipStream_t st = s.stream;
        if (prev >= 0) VX_HIP(hipStreamWaitEvent(st, c->slots[prev].copied, 0));
        VX_HIP(hipMemcpyAsync(s.d_arena, s.h_meta, std::min<uint64_t>(s.arena_cap, (uint64_t)s.cap * 85),
                              hipMemcpyHostToDevice, st));
        VX_HIP(hipMemcpyAsync(s.d_expected, s.h_expected, 20, hipMemcpyHostToDevice, st));
        VX_HIP(hipEventRecord(s.copied, st));
        hipError_t e = vx::launch_uniform(s.d_arena, kAlign, 64, 1, s.d_digests, s.d_expected, s.d_matched, st,
                                          vx::kUniformDefault, nullptr);
        if (e == hipSuccess) {
            s.h_offsets[0] = 0;
            s.h_lens[0] = 64;
            VX_HIP(hipMemcpyAsync(s.d_offsets, s.h_offsets, 8, hipMemcpyHostToDevice, st));
            VX_HIP(hipMemcpyAsync(s.d_lens, s.h_lens, 4, hipMemcpyHostToDevice, st));
            e = vx::launch_ragged(s.d_arena, s.d_offsets, s.d_lens, nullptr, 1, s.d_digests, s.d_expected,
                                  s.d_matched, st, vx::kUniformDefault, nullptr);
        }
        if (e != hipSuccess) return hip_fail(e, "vx_create: warm-up launch");
        VX_HIP(hipMemcpyAsync(s.h_digests, s.d_digests, 20, hipMemcpyDeviceToHost, st));
        VX_HIP(hipMemcpyAsync(s.h_matched, s.d_matched, 1, hipMemcpyDeviceToHost, st));
        VX_HIP(hipEventRecord(s.done, st));
        prev = si;
    }
    for (auto& s : c->slots) VX_HIP(hipStreamSynchronize(s.stream));
    c->last_launched = prev;
    return 0;
}

// A failed launch leaves a slot half-enqueued: the context turns sticky and
// every later call reports the error (vx_destroy still cleans up).
int launch_slot(vx_ctx* c, int si) {
#ifdef VX_TEST_HOOKS
    if (c->fail_launch_after >= 0 && c->fail_launch_after-- == 0)
        return c->sticky = fail(VX_EDEVICE, "launch: injected device failure (vx_tuning_fail_launch_after)");
#endif
    const int rc = launch_slot_impl(c, si);
    if (rc) c->sticky = rc;
    return rc;
}

// Every eligible slot goes zero-copy: the kernel beats gather + hash
// everywhere measured (profiles/r03/zero_copy/).  Full async slots (round-3 A/B, alternating
// runs of async_probe, one registered mmap per buffer): 16 KiB 33 -> 48
// GiB/s, 256 / 512 KiB 47.8 -> 48.8 / 48.1 -> 49.0, 1 / 2 / 4 MiB 44 -> 48 /
// 34 -> 44 / 30 -> 35.  Small, latency-bound batches (round-3 loop-latency A/B,
// 32-piece batches) only in the three-wave form: download-loop p50 at 32 KiB
// 0.68 ms against 0.70, 256 KiB 3.75 against 3.75, 2 MiB 26.6 against 27.7.

// The loader wave takes the loads off the producer, so the chain reading host
// memory runs at 0.78 us per block instead of 0.83-0.86 (tools/zc_chain_probe
// .py): latency-bound batches then finish 7-9 % sooner (p50 at 256 KiB 3.75
// ms against 4.13, 2 MiB 26.7 against 28.8).  On full slots, where PCIe
// binds, it ran 2-4 % behind the pair (256 KiB streamed 49.1 against 50.9
// GiB/s; ab_loader3.jsonl), so those keep the pair.
bool zc_loader_wins(uint32_t n) { return n < kZcMinPieces; }

int launch_slot_impl(vx_ctx* c, int si) {
    Slot& s = c->slots[si];
    if (c->filling == si) {
        c->filling = -1;
        c->flush_pending = false;
    }
    if (s.n == 0) {
        s.state = Slot::FREE;
        return 0;
    }
    hipStream_t cs = s.stream;
    // Zero-copy slot: every piece is read by the hash kernel itself, so no
    // bytes cross PCIe ahead of it and nothing waits for the copy chain.
    // Any slot qualifies, async or inside a host batch (vx_hash.h).
    const bool zc = s.gtiles && s.all_mapped && c->cfg.zero_copy;
    stage_copies(s);
    if (!zc)
        if (int rc = chain_h2d(c, si)) return rc;
    for (const DirectRun& r : s.druns)
        VX_HIP(hipMemcpyAsync(s.d_arena + r.lo, r.host, r.hi - r.lo, hipMemcpyHostToDevice, cs));
    for (const Run& r : s.runs)
        VX_HIP(hipMemcpyAsync(s.d_arena + r.lo, s.h_stage + r.lo, r.hi - r.lo, hipMemcpyHostToDevice, cs));
    const uint32_t n = s.n;
    if (!zc && (!s.uniform || s.gtiles)) {
        VX_HIP(hipMemcpyAsync(s.d_offsets, s.h_offsets, (size_t)n * 8, hipMemcpyHostToDevice, cs));
        VX_HIP(hipMemcpyAsync(s.d_lens, s.h_lens, (size_t)n * 4, hipMemcpyHostToDevice, cs));
    }
    if (zc) {
        VX_HIP(hipMemcpyAsync(s.d_lens, s.h_lens, (size_t)n * 4, hipMemcpyHostToDevice, cs));
        VX_HIP(hipMemcpyAsync(s.d_src, s.h_src, (size_t)n * 8, hipMemcpyHostToDevice, cs));
    } else if (s.gtiles) {
        VX_HIP(hipMemcpyAsync(s.d_src, s.h_src, (size_t)n * 8, hipMemcpyHostToDevice, cs));
        VX_HIP(hipMemcpyAsync(s.d_tfirst, s.h_tfirst, (size_t)(n + 1) * 4, hipMemcpyHostToDevice, cs));
        // Slots of long pieces (>= 2 MiB on average) hash with a few
        // chain-bound pairs that barely touch HBM, so the gather may use 128
        // workgroups: async 2 / 4 MiB pieces 39.8 -> 43.2 / 35.8 -> 39.6 GiB/s.
        // With shorter pieces the hash kernels compete and 128 cost up to 10 %
        // (1 MiB: -2 %).
        const uint32_t grid = s.bytes >= (uint64_t)n << 21 ? 128u : 0u;
        hipError_t e = vx::launch_gather(s.d_src, s.d_offsets, s.d_lens, s.d_tfirst, n, s.gtiles, s.d_arena, cs, grid);
        if (e != hipSuccess) return hip_fail(e, "gather launch");
        c->stats.gather_tiles += s.gtiles;
    }
    if (s.use_table)
        VX_HIP(hipMemcpyAsync(s.d_pidx, s.h_pidx, (size_t)n * 4, hipMemcpyHostToDevice, cs));
    else if (s.has_expected)
        VX_HIP(hipMemcpyAsync(s.d_expected, s.h_expected, (size_t)n * 20, hipMemcpyHostToDevice, cs));
    const uint8_t* d_exp = s.use_table ? c->d_table : (s.has_expected ? s.d_expected : nullptr);
    const uint32_t* d_row = s.use_table ? s.d_pidx : nullptr;
    VX_HIP(hipEventRecord(s.copied, cs));
    mark_launched(c, si);
    hipError_t e;
    if (zc) {
        const bool loader = zc_loader_wins(n);
        e = vx::launch_zero_copy(s.d_src, s.d_lens, n, s.d_digests, d_exp, s.d_matched, loader, s.stream, d_row);
        c->stats.zero_copy_slots++;
        c->stats.zero_copy_loader_slots += loader;
    } else if (s.uniform) {
        const uint32_t len = s.h_lens[0];
        const uint64_t stride = align_up(std::max<uint32_t>(len, 1), kAlign);
        e = vx::launch_uniform(s.d_arena, stride, len, n, s.d_digests, d_exp, s.d_matched, s.stream,
                               vx::kUniformDefault, d_row);
    } else {
        uint64_t max_len = 0, total = 0;
        for (uint32_t i = 0; i < n; ++i) {
            max_len = std::max<uint64_t>(max_len, s.h_lens[i]);
            total += s.h_lens[i];
        }
        e = vx::launch_ragged(s.d_arena, s.d_offsets, s.d_lens, nullptr, n, s.d_digests, d_exp, s.d_matched,
                              s.stream, vx::plan_ragged(n, max_len, total), d_row);
    }
    if (e != hipSuccess) return hip_fail(e, "kernel launch");
    VX_HIP(hipMemcpyAsync(s.h_digests, s.d_digests, (size_t)n * 20, hipMemcpyDeviceToHost, s.stream));
    if (s.has_expected)
        VX_HIP(hipMemcpyAsync(s.h_matched, s.d_matched, n, hipMemcpyDeviceToHost, s.stream));
    VX_HIP(hipEventRecord(s.done, s.stream));
    s.state = Slot::INFLIGHT;
    s.seq = c->seq++;
    c->stats.batches++;
    return 0;
}

// Batch latency: first piece queued -> results harvested, into the log2
// histogram of vx_stats.
void record_batch_latency(vx_ctx* c, std::chrono::steady_clock::time_point t_open) {
    const auto us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t_open);
    const uint64_t v = (uint64_t)std::max<int64_t>(0, us.count());
    vx_stats& st = c->stats;
    st.batch_latency_count++;
    st.batch_latency_sum_us += v;
    st.batch_latency_max_us = std::max(st.batch_latency_max_us, v);
    int k = 0;
    while (k + 1 < VX_STATS_HIST && (v >> (k + 1)) != 0) ++k;
    st.batch_latency_hist[k]++;
}

void harvest(vx_ctx* c, Slot& s) {
    uint64_t bytes = 0, bad = 0;
    for (uint32_t i = 0; i < s.n; ++i) {
        vx_completion r{};
        r.tag = s.tags[i];
        r.matched = s.has_expected ? s.h_matched[i] : 0;
        std::memcpy(r.digest, s.h_digests + (size_t)i * 20, 20);
        c->done.push_back(r);
        bytes += s.h_lens[i];
        bad += s.has_expected && !r.matched;
    }
    if (s.n) {
        c->stats.pieces_completed += s.n;
        if (c->harvest_counts_mismatches) c->stats.pieces_mismatched += bad;
        c->stats.bytes_completed += bytes;
        record_batch_latency(c, s.t_open);
    }
    reset_fill(s);
    s.state = Slot::FREE;
}

// Harvest finished slots (oldest first).  block=true waits for the oldest.
int reap(vx_ctx* c, bool block_oldest) {
    std::vector<int> order;
    for (int i = 0; i < (int)c->slots.size(); ++i)
        if (c->slots[i].state == Slot::INFLIGHT) order.push_back(i);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return c->slots[a].seq < c->slots[b].seq; });
    bool first = true;
    for (int i : order) {
        Slot& s = c->slots[i];
        hipError_t q = (block_oldest && first) ? hipEventSynchronize(s.done) : hipEventQuery(s.done);
        first = false;
        if (q == hipSuccess) {
            harvest(c, s);
        } else if (q != hipErrorNotReady) {
            c->sticky = hip_fail(q, "batch failed on device");
            return c->sticky;
        }
    }
    return 0;
}

// A flush may launch now if, after it, a slot is still free to fill (with a
// single slot: if nothing is in flight).
bool may_launch_now(const vx_ctx* c) {
    int inflight = 0;
    for (const Slot& s : c->slots) inflight += s.state == Slot::INFLIGHT;
    return inflight < std::max(1, (int)c->slots.size() - 1);
}

// may_wait = false (an async submit with refuse_when_full): harvest what has
// finished without blocking, and if no slot is free then, VX_EBUSY.
int acquire_filling(vx_ctx* c, bool may_wait = true) {
    if (c->filling >= 0) return c->filling;
    for (int attempt = 0;; ++attempt) {
        for (int i = 0; i < (int)c->slots.size(); ++i) {
            if (c->slots[i].state == Slot::FREE) {
                reset_fill(c->slots[i]);
                c->slots[i].state = Slot::FILLING;
                c->filling = i;
                return i;
            }
        }
        if (!may_wait) {
            if (attempt > 0) {
                c->stats.submits_refused++;
                return fail(VX_EBUSY, "vx_submit: every slot in flight (refuse_when_full)");
            }
            if (int rc = reap(c, /*block_oldest=*/false)) return rc;
            continue;
        }
        const auto t0 = std::chrono::steady_clock::now();
        int rc = reap(c, /*block_oldest=*/true);
        c->stats.submit_stall_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                        std::chrono::steady_clock::now() - t0).count();
        if (rc) return rc;
    }
}

// piece_row < 0: compare with `expected` (may be NULL); piece_row >= 0:
// compare with row piece_row of the device piece table.
int submit_impl(vx_ctx* c, uint64_t tag, const uint8_t* data, uint32_t len, const uint8_t* expected,
                int64_t piece_row = -1) {
    if (c->sticky) return c->sticky;
    if (!data && len) return fail(VX_EINVAL, "vx_submit: data is NULL");
    if (len > c->cfg.max_piece_len) return fail(VX_ERANGE, "vx_submit: piece longer than max_piece_len");
#ifdef VX_TEST_HOOKS
    if (c->fail_submit_after >= 0 && c->fail_submit_after-- == 0)
        return fail(VX_ENOMEM, "vx_submit: injected failure (vx_tuning_fail_submit_after)");
#endif
    const bool table = piece_row >= 0;
    const bool may_wait = !c->cfg.refuse_when_full || c->bulk;  // host batches always wait
    int si = acquire_filling(c, may_wait);
    if (si < 0) return si;
    Slot* s = &c->slots[si];
    uint64_t off = align_up(s->bytes, kAlign);
    // a slot holds either table-indexed or explicit-digest pieces
    if (s->n == s->cap || off + len > s->arena_cap || (s->n && s->use_table != table)) {
        int rc = launch_slot(c, si);
        if (rc) return rc;
        si = acquire_filling(c, may_wait);
        if (si < 0) return si;
        s = &c->slots[si];
        off = 0;
    }
    const uint32_t i = s->n;
    const uint8_t* dev = nullptr;
    s->h_src[i] = 0;
    if (i == 0) s->t_open = std::chrono::steady_clock::now();
    if (len && (reinterpret_cast<uintptr_t>(data) & 15) == 0 && is_registered(c, data, len, &dev)) {
        // Registered, 16-byte aligned: the launch's gather kernel pulls it
        // through the range's device mapping.
        s->h_src[i] = reinterpret_cast<uint64_t>(dev);
        s->gtiles += vx::gather_tiles(len);
    } else if (len) {
        // all_mapped is cleared below, once the piece is certainly queued: a
        // refused piece (VX_ENOMEM from ensure_stage) must not take the rest
        // of the slot off the zero-copy path.
        if (is_registered(c, data, len)) {
            // Pinned source: DMA straight from the caller's buffer at launch;
            // pieces adjacent in host memory AND in the arena share one copy.
            if (!s->druns.empty() && s->druns.back().hi == off &&
                s->druns.back().host + (s->druns.back().hi - s->druns.back().lo) == data)
                s->druns.back().hi = off + len;
            else
                s->druns.push_back(DirectRun{data, off, off + len});
        } else {
            if (int rc = ensure_stage(c, *s)) return rc;
            c->stats.staged_bytes += len;
            if (c->bulk) {  // a host batch: copied in parallel at launch (stage_copies)
                s->staged.push_back(StageCopy{data, off, len});
                s->staged_bytes += len;
            } else {
                std::memcpy(s->h_stage + off, data, len);
            }
            if (!s->runs.empty() && s->runs.back().hi == off)
                s->runs.back().hi = off + len;
            else if (!s->runs.empty() && align_up(s->runs.back().hi, kAlign) == off)
                s->runs.back().hi = off + len;  // alignment gap travels too
            else
                s->runs.push_back(Run{off, off + len});
        }
        s->all_mapped = false;
    }
    s->h_offsets[i] = off;
    s->h_lens[i] = len;
    s->h_tfirst[i + 1] = s->gtiles;
    // Equal lengths at 256-byte aligned back-to-back offsets are a uniform
    // batch: offset(i) = i * align_up(len, 256) (the uniform kernel's layout).
    if (i > 0 && len != s->h_lens[0]) s->uniform = false;
    if (table) {
        s->h_pidx[i] = (uint32_t)piece_row;
        s->use_table = true;
        s->has_expected = true;
    } else if (expected) {
        std::memcpy(s->h_expected + (size_t)i * 20, expected, 20);
        if (i > 0 && !s->has_expected) {
            // earlier pieces of this batch had no expected digest: they get
            // matched = 0 against a zero table, which nobody reads.
            std::memset(s->h_expected, 0, (size_t)i * 20);
        }
        s->has_expected = true;
    } else if (s->has_expected) {
        std::memset(s->h_expected + (size_t)i * 20, 0, 20);
    }
    s->tags.push_back(tag);
    s->n = i + 1;
    s->bytes = off + std::max<uint32_t>(len, 1);
    c->pending++;
    if (s->n >= c->cfg.batch_pieces && !c->bulk) {
        if (int rc = launch_slot(c, si)) {
            // One rule for every submit (vx_hash.h): a non-zero return means
            // the piece was NOT taken.  The launch failed (the context is now
            // sticky), so this piece leaves the batch again and goes back to
            // the caller with the error; the rest of the slot stays pending and
            // is what the caller recovers after vx_poll reports the failure.
            s->tags.pop_back();
            s->n = i;
            c->pending--;
            return rc;
        }
    }
    return 0;
}

}  // namespace

extern "C" {

int vx_abi_version(void) { return VX_ABI_VERSION; }

const char* vx_last_error(void) { return g_err.c_str(); }

const char* vx_strerror(int code) {
    switch (code) {
        case VX_OK: return "ok";
        case VX_EINVAL: return "invalid argument";
        case VX_ENOMEM: return "out of memory";
        case VX_ERANGE: return "piece longer than max_piece_len";
        case VX_ENODEV: return "no such device";
        case VX_EDEVICE: return "HIP runtime error";
        case VX_EBUSY: return "busy: work in flight";
        default: return "unknown error";
    }
}

int vx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void vx_config_default(vx_config* cfg, uint32_t max_piece_len) {
    if (!cfg) return;
    cfg->device = 0;
    cfg->max_piece_len = max_piece_len;
    cfg->slots = 4;
    // Throughput of the async path is bytes in flight / batch latency, and a
    // batch's latency is its longest piece's chain (~28 ms at 2 MiB: one lane
    // hashes ~74 MB/s), so slots grow with the piece length: 512 pieces each,
    // 128 MiB to 2 GiB of HBM.  128 pieces per slot held only ~512 lanes in
    // flight over 4 slots; 512 took async 2 MiB pieces 25.7 -> 32.8 GiB/s and
    // 4 MiB 22.3 -> 27.1 (profiles/r01/async/slot_sweep.jsonl).  (The pinned
    // stage is only allocated for unregistered pieces; keeping it at 128 MiB
    // for short pieces keeps their staging memcpy cache-friendly: 256 MiB
    // slots halved the unregistered 16 KiB rate, async_probe.)
    const uint64_t piece = align_up(std::max<uint32_t>(max_piece_len, 1), kAlign);
    cfg->slot_bytes = std::max(piece, std::min<uint64_t>(2ull << 30, std::max<uint64_t>(128ull << 20, piece * 512)));
    cfg->batch_pieces = (uint32_t)std::min<uint64_t>(65536, cfg->slot_bytes / align_up(std::max<uint32_t>(max_piece_len, 1), kAlign));
    cfg->zero_copy = 1;
    cfg->direct_io = 1;
    cfg->batch_chunk = 64 * 1024;
    cfg->verify_chunk = 0;         // per call: verify_chunk_for
    cfg->verify_cold_chunk = 0;
    cfg->verify_ramp = 1;
    cfg->refuse_when_full = 0;
}

int vx_create(const vx_config* cfg, vx_ctx** out) {
    if (!cfg || !out) return fail(VX_EINVAL, "vx_create: NULL argument");
    *out = nullptr;
    if (cfg->max_piece_len == 0 || cfg->slots == 0 || cfg->batch_pieces == 0)
        return fail(VX_EINVAL, "vx_create: max_piece_len, slots and batch_pieces must be > 0");
    if (cfg->slot_bytes < cfg->max_piece_len) return fail(VX_EINVAL, "vx_create: slot_bytes < max_piece_len");
    if (cfg->zero_copy > 1 || cfg->direct_io > 1 || cfg->refuse_when_full > 1)
        return fail(VX_EINVAL, "vx_create: zero_copy, direct_io and refuse_when_full are 0 or 1");
    if (cfg->verify_ramp > 5) return fail(VX_EINVAL, "vx_create: verify_ramp must be 0..5");
    if ((cfg->batch_chunk && (cfg->batch_chunk < 4096 || cfg->batch_chunk % 4096)) ||
        (cfg->verify_chunk && (cfg->verify_chunk < 4096 || cfg->verify_chunk % 4096)) ||
        (cfg->verify_cold_chunk && (cfg->verify_cold_chunk < 4096 || cfg->verify_cold_chunk % 4096)))
        return fail(VX_EINVAL, "vx_create: chunk sizes must be 0 or multiples of 4096");
    // At most 1 GiB: a wrapped negative value from a binding is a huge
    // multiple of 4096.  (A chunk larger than a slot's arena is
    // legal: those calls take the whole-piece path.)
    constexpr uint32_t kMaxChunk = 1u << 30;
    if (cfg->batch_chunk > kMaxChunk || cfg->verify_chunk > kMaxChunk || cfg->verify_cold_chunk > kMaxChunk)
        return fail(VX_EINVAL, "vx_create: chunk sizes must be at most 1 GiB");
    const int ndev = vx_device_count();
    if (cfg->device < 0 || cfg->device >= ndev) return fail(VX_ENODEV, "vx_create: no such HIP device");
    vx_ctx* c = new (std::nothrow) vx_ctx();
    if (!c) return fail(VX_ENOMEM, "vx_create: out of host memory");
    c->cfg = *cfg;
    int rc = set_device(c);
    if (!rc) {
        c->slots.resize(cfg->slots);
        for (auto& s : c->slots) {
            rc = alloc_slot(s, cfg->slot_bytes, slot_capacity(cfg));
            if (rc) break;
        }
    }
    if (!rc) rc = warm_slots(c);
    if (rc) {
        for (auto& s : c->slots) free_slot_mem(s);
        delete c;
        return rc;
    }
    *out = c;
    return 0;
}

int vx_destroy(vx_ctx* c) {
    if (!c) return 0;
    int rc = c->sticky ? 0 : vx_drain(c, 0);
    set_device(c);
    // A failed (sticky) context skipped the drain: batches may still be
    // running, and a gather kernel may still read registered host memory.
    // Wait for every stream before unregistering anything, so the caller can
    // return in-flight buffers to its pool as soon as this call returns.
    for (auto& s : c->slots)
        if (s.stream) (void)hipStreamSynchronize(s.stream);
    // the re-verify's data copies run on the copy stream: a failed call may
    // have left one queued that still reads a stage or writes an arena
    if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
    for (auto& r : c->registered) (void)hipHostUnregister(reinterpret_cast<void*>(r.first));
    for (auto& s : c->slots) free_slot_mem(s);
    if (c->d_table) (void)hipFree(c->d_table);
    if (c->d_chunk_rows) (void)hipFree(c->d_chunk_rows);
    if (c->chunk_prev) (void)hipEventDestroy(c->chunk_prev);
    for (hipEvent_t e : c->copy_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->anchor_ev) (void)hipEventDestroy(c->anchor_ev);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    delete c;
    return rc;
}

int vx_register_host_buffer(vx_ctx* c, void* ptr, size_t len) {
    if (!c || !ptr || !len) return fail(VX_EINVAL, "vx_register_host_buffer: bad argument");
    const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
    auto it = c->registered.lower_bound(a);
    if (it != c->registered.end() && it->first < a + len) return fail(VX_EINVAL, "overlapping registration");
    if (it != c->registered.begin()) {
        auto p = std::prev(it);
        if (p->first + p->second.len > a) return fail(VX_EINVAL, "overlapping registration");
    }
    int rc = set_device(c);
    if (rc) return rc;
    VX_HIP(hipHostRegister(ptr, len, hipHostRegisterMapped));
    void* dev = nullptr;
    if (hipHostGetDevicePointer(&dev, ptr, 0) != hipSuccess || !dev) {
        (void)hipHostUnregister(ptr);
        return fail(VX_EDEVICE, "vx_register_host_buffer: no device mapping");
    }
    c->registered[a] = vx_ctx::Reg{len, static_cast<uint8_t*>(dev)};
    c->registered_at[a] = vx_ctx::Reg{len, static_cast<uint8_t*>(dev)};
    return 0;
}

int vx_unregister_host_buffer(vx_ctx* c, void* ptr) {
    if (!c || !ptr) return fail(VX_EINVAL, "vx_unregister_host_buffer: bad argument");
    auto it = c->registered.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == c->registered.end()) return fail(VX_EINVAL, "pointer was not registered");
    if (c->pending) return fail(VX_EBUSY, "unregister with pieces in flight");
    int rc = set_device(c);
    if (rc) return rc;
    VX_HIP(hipHostUnregister(ptr));
    c->registered.erase(it);
    c->registered_at.erase(reinterpret_cast<uintptr_t>(ptr));
    return 0;
}

int vx_submit(vx_ctx* c, uint64_t tag, const uint8_t* data, uint32_t len, const uint8_t* expected) {
    if (!c) return fail(VX_EINVAL, "vx_submit: NULL context");
    int rc = set_device(c);
    if (rc) return rc;
    return submit_impl(c, tag, data, len, expected);
}

int vx_set_piece_table(vx_ctx* c, const uint8_t* table, uint32_t n_pieces) {
    if (!c || (n_pieces && !table)) return fail(VX_EINVAL, "vx_set_piece_table: bad argument");
    if (c->pending || c->filling >= 0) return fail(VX_EBUSY, "vx_set_piece_table: pieces in flight");
    int rc = set_device(c);
    if (rc) return rc;
    if (c->d_table) (void)hipFree(c->d_table);
    c->d_table = nullptr;
    c->n_table = 0;
    if (!n_pieces) return 0;
    if (hipMalloc(&c->d_table, (size_t)n_pieces * 20) != hipSuccess)
        return fail(VX_ENOMEM, "vx_set_piece_table: device allocation failed");
    VX_HIP(hipMemcpy(c->d_table, table, (size_t)n_pieces * 20, hipMemcpyHostToDevice));
    c->n_table = n_pieces;
    return 0;
}

int vx_submit_piece(vx_ctx* c, uint64_t tag, const uint8_t* data, uint32_t len, uint32_t piece_index) {
    if (!c) return fail(VX_EINVAL, "vx_submit_piece: NULL context");
    if (piece_index >= c->n_table) return fail(VX_EINVAL, "vx_submit_piece: piece_index outside the piece table");
    int rc = set_device(c);
    if (rc) return rc;
    return submit_impl(c, tag, data, len, nullptr, (int64_t)piece_index);
}

// Launch the filling slot unless that would leave no slot free for the next
// submit: then the slot stays open and keeps collecting pieces, and vx_poll
// launches it as soon as a batch completes.  So under load batches grow
// instead of the event-loop thread blocking in vx_submit for a whole batch
// (DESIGN.md §6.5).
int vx_flush(vx_ctx* c) {
    if (!c) return fail(VX_EINVAL, "vx_flush: NULL context");
    if (c->sticky) return c->sticky;
    if (c->filling < 0 || c->slots[c->filling].n == 0) return 0;
    int rc = set_device(c);
    if (rc) return rc;
    if ((rc = reap(c, false))) return rc;
    if (!may_launch_now(c)) {
        c->flush_pending = true;
        return 0;
    }
    return launch_slot(c, c->filling);
}

int64_t vx_poll(vx_ctx* c, vx_completion* out, size_t max) {
    if (!c || (!out && max)) return fail(VX_EINVAL, "vx_poll: bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    if (c->sticky) {
        // Failed context: hand out every result the device did produce (batches
        // that finished, harvested now or earlier), then the error.  The tags
        // never returned are the pieces to re-hash elsewhere.
        const int sticky = c->sticky;
        (void)reap(c, false);
        c->sticky = sticky;
        if (c->done.empty()) return sticky;
    } else {
        rc = reap(c, false);
        if (rc) return rc;
        if (c->flush_pending && c->filling >= 0 && may_launch_now(c) && (rc = launch_slot(c, c->filling))) return rc;
    }
    size_t k = 0;
    while (k < max && !c->done.empty()) {
        out[k++] = c->done.front();
        c->done.pop_front();
    }
    c->pending -= k;
    return (int64_t)k;
}

int vx_drain(vx_ctx* c, uint32_t timeout_ms) {
    if (!c) return fail(VX_EINVAL, "vx_drain: NULL context");
    if (c->sticky) return c->sticky;
    int rc = set_device(c);
    if (rc) return rc;
    if (c->filling >= 0 && (rc = launch_slot(c, c->filling))) return rc;  // forced, unlike vx_flush
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        bool any = false;
        for (auto& s : c->slots) any |= s.state == Slot::INFLIGHT;
        if (!any) return 0;
        if (timeout_ms == 0) {
            rc = reap(c, true);
        } else {
            rc = reap(c, false);
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms))
                return fail(VX_EBUSY, "vx_drain: timeout");
            std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
        if (rc) return rc;
    }
}

uint64_t vx_pending(const vx_ctx* c) { return c ? c->pending : 0; }

// Bulk re-verify from disk (include/vx_hash.h).
//
// Pieces shorter than two chunks (verify_chunk_for): the reader threads pread each slot's pieces
// straight into that slot's pinned stage (segments back to back,
// file_store.rs:240-298 byte ranges) and the slot launches while the next free
// slot is read.  Longer pieces: resumable chunked hashing — round k reads
// chunk k of every piece of a window into a slot, and the chunk kernel
// continues each piece's 20-byte SHA-1 state from round k-1, so PCIe moves
// round k+1 while the GPU compresses round k and no launch waits on a whole
// multi-MiB chain.  Completions are consumed here; they never reach vx_poll.
}  // extern "C" (the helpers below are C++ templates)

namespace {

struct FileVerify {
    vx_ctx* c;
    const uint8_t* expected;
    uint8_t* matched_out;
    std::vector<uint8_t>& bad;
    uint64_t done = 0;

    void consume() {
        while (!c->done.empty()) {
            const vx_completion& r = c->done.front();
            matched_out[r.tag] = (r.matched && !bad[r.tag]) ? 1 : 0;
            c->stats.pieces_mismatched += !r.matched && !bad[r.tag];  // I/O errors count in io_errors only
            c->done.pop_front();
            ++done;
        }
    }
    int free_slot() {
        for (;;) {
            bool inflight = false;
            for (int k = 0; k < (int)c->slots.size(); ++k) {
                if (c->slots[k].state == Slot::FREE) return k;
                inflight |= c->slots[k].state == Slot::INFLIGHT;
            }
            if (!inflight) return fail(VX_EDEVICE, "vx_verify_files: no slot to wait for");
            int rc = reap(c, true);
            consume();
            if (rc) return rc;
        }
    }
};

// Re-verify chunk size for `count` pieces: 256 KiB when
// every piece's chunk fits one slot arena (a single window of rounds), else
// 128 KiB.  A call split into windows ends on its last, smaller window, whose
// rounds are chain-bound; measured (profiles/r01/reverify/policy*.json):
// 1 MiB x 2,774 pieces 43.6 -> 46.8 GiB/s at 128 KiB, 256 KiB x 11,093 pieces
// 37.5 (whole-piece slots) -> 45.0, 2 MiB x 1,387 best at 256 KiB + ramp.
uint64_t verify_chunk_for(const vx_ctx* c, uint64_t count) {
    if (c->cfg.verify_chunk) return c->cfg.verify_chunk;
    constexpr uint64_t big = 256 * 1024, small = 128 * 1024;
    return count * big <= c->slots[0].arena_cap && count <= c->slots[0].cap ? big : small;
}

// Re-verify reads run this many slots (whole pieces) or rounds (chunks)
// ahead of the one being enqueued, bounded by the slots.
constexpr size_t kReadahead = 2;

// Both verify pieces [first, end) of an n-piece torrent; tags, bad[] and
// matched_out are indexed from `first`.  Both queue reads up to kReadahead
// slots ahead of the slot being launched (see verify_chunked).
int verify_whole(FileVerify& fv, vx_files::Readers& rd, uint64_t n, uint32_t pl, uint64_t total, uint64_t first,
                 uint64_t end) {
    vx_ctx* c = fv.c;
    const uint64_t stride = align_up(pl, kAlign);
    const uint64_t last_len = total - (n - 1) * (uint64_t)pl;
    const size_t nslots = c->slots.size();
    const size_t depth = nslots > 1 ? std::min<size_t>(kReadahead, nslots - 1) : 0;
    std::vector<std::vector<vx_files::ReadItem>> items(nslots);
    struct Queued {
        int si;
        uint64_t ticket;
    };
    std::deque<Queued> q;  // slots read or reading, in piece order, not yet launched
    // Runs of whole pieces inside one file go out as one pread of up to 4 MiB
    // (vx_files::Runs; 16 KiB pieces were pread-bound).
    vx_files::Runs runs = rd.runs(4ull << 20);
    // Ramps: nothing overlaps the first slot's read or the last slot's copy
    // and kernel, so the first slots take 1/2^L, ..., 1/4, 1/2 of a full
    // slot's pieces, the first one <= 64 MiB, and the last full slot's worth
    // is split in halves down to that size (cfg.verify_ramp = 0 turns both
    // off; as for chunks, §6.3).
    const uint64_t cap_full =
        std::min<uint64_t>(c->slots[0].cap, std::max<uint64_t>(1, c->slots[0].arena_cap / stride));
    int ramp = 0;
    while (c->cfg.verify_ramp > 0 && ramp < 8 && (cap_full >> ramp) > 1 && (cap_full >> ramp) * stride > (64ull << 20))
        ++ramp;
    int filled = 0;
    uint64_t next = first;
    int rc = 0;
    while ((next < end || !q.empty()) && !rc) {
        // The slot to launch next may wait for a free slot; later ones take
        // only a slot that is free now.
        while (next < end && q.size() <= depth) {
            int si = -1;
            if (q.empty()) {
                si = fv.free_slot();
                if (si < 0) rc = si;
            } else {
                rc = reap(c, false);
                fv.consume();
                for (int k = 0; k < (int)nslots && !rc; ++k)
                    if (c->slots[k].state == Slot::FREE) {
                        si = k;
                        break;
                    }
            }
            if (rc || si < 0) break;
            Slot& s = c->slots[si];
            reset_fill(s);
            if ((rc = ensure_stage(c, s))) break;
            s.state = Slot::FILLING;  // reserved until launched
            s.t_open = std::chrono::steady_clock::now();
            uint64_t cap = filled < ramp ? std::max<uint64_t>(1, cap_full >> (ramp - filled)) : cap_full;
            const uint64_t rem = end - next, smallest = std::max<uint64_t>(1, cap_full >> ramp);
            if (ramp > 0 && rem <= cap && rem > smallest) cap = std::max(smallest, (rem + 1) / 2);
            ++filled;
            const uint64_t lo = next, hi = std::min<uint64_t>(end, next + cap);
            auto& it = items[si];
            it.clear();
            for (uint64_t i = lo; i < hi; ++i) {
                const uint32_t len = (uint32_t)(i == n - 1 ? last_len : pl);
                const uint32_t k = (uint32_t)(i - lo);
                runs.add(it, s.h_stage + k * stride, i, len);
                s.h_offsets[k] = k * stride;
                s.h_lens[k] = len;
                if (len != s.h_lens[0]) s.uniform = false;
                std::memcpy(s.h_expected + (size_t)k * 20, fv.expected + 20 * i, 20);
                s.tags.push_back(i - first);
            }
            s.n = (uint32_t)(hi - lo);
            s.has_expected = true;
            s.bytes = (hi - lo - 1) * stride + s.h_lens[s.n - 1];
            s.runs.push_back(Run{0, s.bytes});
            q.push_back(Queued{si, rd.submit(it)});
            next = hi;
        }
        if (rc || q.empty()) break;
        const Queued head = q.front();
        q.pop_front();
        rd.wait(head.ticket);
        rc = launch_slot(c, head.si);
        if (!rc) rc = reap(c, false);
        fv.consume();
    }
    rd.wait();  // error path: no read may still target a stage
    for (auto& sl : c->slots)  // slots read but never launched (error path)
        if (sl.state == Slot::FILLING) {
            reset_fill(sl);
            sl.state = Slot::FREE;
        }
    return rc;
}

// Resumable chunk pipeline, shared by the file
// re-verify and strided host batches.  The call owns per-piece device rows
// (chaining state, expected digest, digest, verdict).  Each round is one slot:
// its H2D joins the copy chain across slots (chain_h2d), and its kernel waits
// for the previous round of the same window (state dependency) through
// `prev_kernel`, so PCIe moves round k+1 while the GPU compresses round k.
struct ChunkPipe {
    vx_ctx* c;
    uint64_t cnt = 0;
    uint64_t bytes = 0;  // the call's piece bytes (vx_stats)
    uint32_t* d_states = nullptr;
    uint8_t *d_exp = nullptr, *d_dig = nullptr, *d_match = nullptr;
    hipEvent_t prev_kernel = nullptr;
    bool have_prev = false;
    // Set (use_copy_stream): every round's H2D goes on the context's copy
    // stream, its kernel on the slot's stream after a wait on the round's
    // `copied` event.  Two slot streams can share one hardware queue (HIP maps
    // streams onto GPU_MAX_HW_QUEUES = 4), and a copy queued behind the other
    // slot's kernel there waited for that kernel: 5-7 ms of idle PCIe per
    // warm linux-mint call with 4-6 slots (profiles/r05/gaps/).
    hipStream_t cs = nullptr;
    // Set by a copy_data that records a timing event right after its copy on
    // the copy stream: the slot's stream waits on that one instead of a
    // separate `copied` marker (each marker between two copies on one stream
    // costs the copy engine ~15 us; 36 rounds of 8 MiB pieces add up).
    hipEvent_t copy_end = nullptr;

    explicit ChunkPipe(vx_ctx* ctx) : c(ctx) {}

    int use_copy_stream() {
        if (!c->copy_stream) {
            int least = 0, greatest = 0;
            if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
                hipStreamCreateWithPriority(&c->copy_stream, hipStreamNonBlocking, greatest) != hipSuccess) {
                c->copy_stream = nullptr;
                return fail(VX_EDEVICE, "chunk rounds: copy stream creation failed");
            }
        }
        cs = c->copy_stream;
        return 0;
    }
    ~ChunkPipe() { release(); }
    ChunkPipe(const ChunkPipe&) = delete;
    ChunkPipe& operator=(const ChunkPipe&) = delete;

    // expected: count x 20 bytes or NULL (digests only).
    int open(uint64_t count, const uint8_t* expected, const char* who) {
        cnt = count;
        if (c->chunk_rows_cap < count) {
            if (c->d_chunk_rows) (void)hipFree(c->d_chunk_rows);
            c->d_chunk_rows = nullptr;
            c->chunk_rows_cap = 0;
            const uint64_t cap = std::max<uint64_t>(count, 4096);
            if (hipMalloc(&c->d_chunk_rows, cap * 61 + 256) != hipSuccess)
                return fail(VX_ENOMEM, std::string(who) + ": device allocation failed");
            c->chunk_rows_cap = cap;
        }
        const uint64_t cap = c->chunk_rows_cap;
        d_states = reinterpret_cast<uint32_t*>(c->d_chunk_rows);
        d_dig = c->d_chunk_rows + cap * 20;
        d_exp = expected ? c->d_chunk_rows + cap * 40 : nullptr;
        d_match = expected ? c->d_chunk_rows + cap * 60 : nullptr;
        if (!c->chunk_prev && hipEventCreateWithFlags(&c->chunk_prev, hipEventDisableTiming) != hipSuccess)
            return fail(VX_EDEVICE, std::string(who) + ": event creation failed");
        prev_kernel = c->chunk_prev;
        if (expected && hipMemcpy(d_exp, expected, cnt * 20, hipMemcpyHostToDevice) != hipSuccess)
            return fail(VX_EDEVICE, std::string(who) + ": expected-table upload failed");
        return 0;
    }

    // A free slot, reaping the oldest round when none is; on_reap runs after
    // every blocking reap (the file path consumes whole-piece completions).
    template <class F>
    int free_slot(F&& on_reap) {
        for (;;) {
            bool inflight = false;
            for (int k = 0; k < (int)c->slots.size(); ++k) {
                if (c->slots[k].state == Slot::FREE) return k;
                inflight |= c->slots[k].state == Slot::INFLIGHT;
            }
            if (!inflight) return fail(VX_EDEVICE, "chunk rounds: no slot to wait for");
            int rc = reap(c, true);
            on_reap();
            if (rc) return rc;
        }
    }
    // A slot that is free now, after polling completions without blocking;
    // -1 in *si when there is none.
    template <class F>
    int try_free_slot(int* si, F&& on_reap) {
        *si = -1;
        const int rc = reap(c, false);
        on_reap();
        if (rc) return rc;
        for (int k = 0; k < (int)c->slots.size(); ++k)
            if (c->slots[k].state == Slot::FREE) {
                *si = k;
                break;
            }
        return 0;
    }

    // Slot si's h_offsets/h_lens/h_pidx/h_poff/h_tlen [0, m) describe the
    // round's lanes; copy_data(slot, stream) enqueues the chunk bytes into the
    // slot arena.  The lane table goes up as ONE copy of the metadata block's
    // head (offsets | chunk offsets | total lens | gather sources | lens |
    // piece rows, alloc_slot), not five: each small H2D is a blit kernel, and
    // five of them put ~0.1 ms between one round's data copy and the next.
    // When copy_data is a plain copy the table follows it, after `copied`, so
    // the next round's data copy (chained on `copied`) need not wait for it;
    // a gather (meta_first) reads d_offsets/d_lens, so the table goes first.
    // continues = the round follows one of the same window.
    template <class F>
    int round(int si, uint32_t m, bool continues, bool meta_first, F&& copy_data) {
        if (cs) return round_cs(si, m, continues, copy_data);
        Slot& s = c->slots[si];
        hipStream_t st = s.stream;
        int rc = chain_h2d(c, si);
        const size_t meta = (size_t)(reinterpret_cast<const uint8_t*>(s.h_pidx + m) - reinterpret_cast<const uint8_t*>(s.h_offsets));
        auto table = [&] {
            if (hipMemcpyAsync(s.d_offsets, s.h_offsets, meta, hipMemcpyHostToDevice, st) != hipSuccess)
                return fail(VX_EDEVICE, "chunk round: H2D failed");
            return 0;
        };
        if (!rc && meta_first) rc = table();
        if (!rc) rc = copy_data(s, st);
        if (!rc && hipEventRecord(s.copied, st) != hipSuccess) rc = fail(VX_EDEVICE, "chunk round: event failed");
        if (!rc && !meta_first) rc = table();
        mark_launched(c, si);
        if (!rc && continues && have_prev && hipStreamWaitEvent(st, prev_kernel, 0) != hipSuccess)
            rc = fail(VX_EDEVICE, "chunk round: stream wait failed");
#ifdef VX_TEST_HOOKS
        if (!rc && c->fail_launch_after >= 0 && c->fail_launch_after-- == 0)
            rc = fail(VX_EDEVICE, "chunk round: injected launch failure (vx_tuning_fail_launch_after)");
#endif
        if (!rc) {
            hipError_t e = vx::launch_chunk(s.d_arena, s.d_offsets, s.d_lens, m, s.d_pidx, s.d_poff, s.d_tlen,
                                            d_states, d_dig, d_exp, d_match, st);
            if (e != hipSuccess) rc = hip_fail(e, "chunk kernel launch");
        }
        if (!rc && (hipEventRecord(prev_kernel, st) != hipSuccess || hipEventRecord(s.done, st) != hipSuccess))
            rc = fail(VX_EDEVICE, "chunk round: event record failed");
        have_prev = true;
        c->stats.chunk_rounds++;
        s.state = Slot::INFLIGHT;
        s.seq = c->seq++;
        s.n = 0;  // nothing to harvest: outputs live in the call's device rows
        if (rc) (void)hipStreamSynchronize(st);  // s.done may be stale: let the queued part finish
        if (!rc) rc = reap(c, false);
        return rc;
    }
    // round() with the data copies on the copy stream, then `copied`; the
    // slot's stream takes the round's small lane table, waits for `copied`
    // and runs the kernel.  The data copies stay in launch order (one stream)
    // back to back, with no host wait and no small table copy between them
    // (on the copy stream each table added ~70 us to every round: 2.6 ms of
    // a 1,024 x 8 MiB call, profiles/r05/gaps/).  A table behind an aliased
    // slot's kernel only waits where the kernel waits anyway (the previous
    // round's state).  The slot is reused only after its `done` (free_slot),
    // so no copy overwrites a stage or arena a kernel still reads.
    template <class F>
    int round_cs(int si, uint32_t m, bool continues, F&& copy_data) {
        Slot& s = c->slots[si];
        hipStream_t st = s.stream;
        const size_t meta = (size_t)(reinterpret_cast<const uint8_t*>(s.h_pidx + m) - reinterpret_cast<const uint8_t*>(s.h_offsets));
        copy_end = nullptr;
        int rc = copy_data(s, cs);
        hipEvent_t copied = copy_end ? copy_end : s.copied;
        if (!rc && copied == s.copied && hipEventRecord(s.copied, cs) != hipSuccess)
            rc = fail(VX_EDEVICE, "chunk round: event failed");
        if (!rc && hipMemcpyAsync(s.d_offsets, s.h_offsets, meta, hipMemcpyHostToDevice, st) != hipSuccess)
            rc = fail(VX_EDEVICE, "chunk round: H2D failed");
        mark_launched(c, si);
        if (!rc && hipStreamWaitEvent(st, copied, 0) != hipSuccess)
            rc = fail(VX_EDEVICE, "chunk round: stream wait failed");
        if (!rc && continues && have_prev && hipStreamWaitEvent(st, prev_kernel, 0) != hipSuccess)
            rc = fail(VX_EDEVICE, "chunk round: stream wait failed");
#ifdef VX_TEST_HOOKS
        if (!rc && c->fail_launch_after >= 0 && c->fail_launch_after-- == 0)
            rc = fail(VX_EDEVICE, "chunk round: injected launch failure (vx_tuning_fail_launch_after)");
#endif
        if (!rc) {
            hipError_t e = vx::launch_chunk(s.d_arena, s.d_offsets, s.d_lens, m, s.d_pidx, s.d_poff, s.d_tlen,
                                            d_states, d_dig, d_exp, d_match, st);
            if (e != hipSuccess) rc = hip_fail(e, "chunk kernel launch");
        }
        if (!rc && (hipEventRecord(prev_kernel, st) != hipSuccess || hipEventRecord(s.done, st) != hipSuccess))
            rc = fail(VX_EDEVICE, "chunk round: event record failed");
        have_prev = true;
        c->stats.chunk_rounds++;
        s.state = Slot::INFLIGHT;
        s.seq = c->seq++;
        s.n = 0;
        if (rc) {
            // Part of the round may be queued (its data copy on the copy
            // stream, the table on the slot's) while s.done was not recorded
            // for it: wait for both here, so no later reuse or free of the
            // stage and arena races a DMA of this round.
            (void)hipStreamSynchronize(cs);
            (void)hipStreamSynchronize(st);
        }
        if (!rc) rc = reap(c, false);
        return rc;
    }
    void end_window() { have_prev = false; }  // windows hold disjoint pieces

    // Wait for every round, then copy verdicts / digests back (either may be
    // NULL).  bad (may be NULL): pieces the caller fails for an I/O error,
    // counted in io_errors and not again as mismatches.
    int finish(uint8_t* matched_out, uint8_t* digests_out, int rc, const uint8_t* bad = nullptr) {
        if (!rc) {
            for (auto& s : c->slots)
                if (s.state == Slot::INFLIGHT && hipEventSynchronize(s.done) != hipSuccess) rc = VX_EDEVICE;
            if (rc) (void)fail(rc, "chunk rounds failed on device");
        }
        if (!rc && matched_out && d_match && hipMemcpy(matched_out, d_match, cnt, hipMemcpyDeviceToHost) != hipSuccess)
            rc = fail(VX_EDEVICE, "verdict D2H failed");
        if (!rc && digests_out && hipMemcpy(digests_out, d_dig, cnt * 20, hipMemcpyDeviceToHost) != hipSuccess)
            rc = fail(VX_EDEVICE, "digest D2H failed");
        if (!rc) {
            c->stats.pieces_completed += cnt;
            c->stats.bytes_completed += bytes;
            if (matched_out && d_match)
                for (uint64_t i = 0; i < cnt; ++i) c->stats.pieces_mismatched += matched_out[i] == 0 && !(bad && bad[i]);
        }
        for (auto& s : c->slots)
            if (s.state == Slot::INFLIGHT) {
                (void)hipEventSynchronize(s.done);
                reset_fill(s);
                s.state = Slot::FREE;
            }
        return rc;
    }

    // finish() for a set of row ranges (the split: this engine's claims):
    // verdicts back for those rows only, and only they count in vx_stats.
    int finish_rows(uint8_t* matched_out, int rc, const uint8_t* bad,
                    const std::vector<std::pair<uint64_t, uint64_t>>& rows) {
        if (!rc) {
            for (auto& s : c->slots)
                if (s.state == Slot::INFLIGHT && hipEventSynchronize(s.done) != hipSuccess) rc = VX_EDEVICE;
            if (rc) (void)fail(rc, "chunk rounds failed on device");
        }
        for (const auto& r : rows) {
            const uint64_t lo = std::min(r.first, cnt), hi = std::min(r.second, cnt);
            if (!rc && matched_out && d_match && hi > lo &&
                hipMemcpy(matched_out + lo, d_match + lo, hi - lo, hipMemcpyDeviceToHost) != hipSuccess)
                rc = fail(VX_EDEVICE, "verdict D2H failed");
        }
        if (!rc) {
            c->stats.bytes_completed += bytes;
            for (const auto& r : rows) {
                c->stats.pieces_completed += r.second - r.first;
                if (matched_out && d_match)
                    for (uint64_t i = r.first; i < r.second; ++i)
                        c->stats.pieces_mismatched += matched_out[i] == 0 && !(bad && bad[i]);
            }
        }
        for (auto& s : c->slots)
            if (s.state == Slot::INFLIGHT) {
                (void)hipEventSynchronize(s.done);
                reset_fill(s);
                s.state = Slot::FREE;
            }
        return rc;
    }

    // The rows and the event belong to the context (freed by vx_destroy);
    // only make sure nothing of this call is still running.
    void release() {
        if (cs) (void)hipStreamSynchronize(cs);  // data copies of this call's rounds
        for (auto& s : c->slots)
            if (s.stream) (void)hipStreamSynchronize(s.stream);
    }
};

// Round boundaries [a, a + len) over a window whose longest piece is L:
// chunks of C, and with `head`/`tail` ramps of depth d (q = C / 2^(d+1)) on
// the first / last C bytes: q, q, 2q, ..., C/2 up front and C/2, ..., 2q, q,
// rest (<= q) at the end, so the first read and the last chain — the parts
// of the pipeline nothing overlaps — shrink to q.  d = 1 is C/4, C/4, C/2.
// Every boundary is a multiple of q (>= 64 bytes for C >= 4 KiB, d <= 5), so
// no non-final chunk ends mid-block.
std::vector<std::pair<uint64_t, uint64_t>> chunk_schedule(uint64_t L, uint64_t C, int head, int tail) {
    std::vector<std::pair<uint64_t, uint64_t>> r;
    const int d = std::max(head, tail);
    const uint64_t q = C >> (d + 1);
    uint64_t a = 0;
    if (L == 0) r.push_back({0, 0});
    const bool ramp = d > 0 && q >= 64 && L >= 2 * C;  // head (ends at C) and tail (from >= C) never overlap
    if (ramp && head) {
        r.push_back({a, q});
        a += q;
        for (uint64_t len = q; len < C; len *= 2) r.push_back({a, len}), a += len;
    }
    // the tail ramp covers the last R bytes, R in (C - q, C]: C/2, ..., q, R - (C - q)
    const uint64_t tail_from = ramp && tail ? (L - C + q - 1) / q * q : L;
    while (a < tail_from) {
        const uint64_t len = std::min(C, tail_from - a);
        r.push_back({a, len});
        a += len;
    }
    if (a < L) {
        for (uint64_t len = C / 2; len >= q; len /= 2) r.push_back({a, len}), a += len;
        r.push_back({a, L - a});
        a = L;
    }
    return r;
}

// The rounds of every window, in order, each read into its own slot by the
// reader pool and then enqueued (H2D + chunk kernel).  Reads run up to
// kReadahead rounds ahead of the round being enqueued (bounded by the slots),
// queued on the pool so the readers never wait for an enqueue: with one round
// of read-ahead the reads and the copy chain were coupled round by round, and
// every round whose read outlasted the previous copy left PCIe idle (the head
// ramp's doubling rounds most of all).  Each round's data
// copy is timed on the GPU (vx_tuning_last_verify).
int verify_chunked(FileVerify& fv, vx_files::Readers& rd, uint64_t n, uint32_t pl, uint64_t total, uint64_t first,
                   uint64_t end, uint64_t C) {
    vx_ctx* c = fv.c;
    const uint64_t last_len = total - (n - 1) * (uint64_t)pl;
    const uint64_t cnt = end - first;
    ChunkPipe cp(c);
    int rc = cp.open(cnt, fv.expected + 20 * first, "vx_verify_files");
    if (!rc && c->verify_copy_stream) rc = cp.use_copy_stream();
    cp.bytes = cnt * (uint64_t)pl - (end == n ? (uint64_t)pl - last_len : 0);
    // windows of W pieces; each window runs its rounds in order
    const Slot& s0 = c->slots[0];
    const uint64_t W = std::max<uint64_t>(1, std::min<uint64_t>(s0.cap, s0.arena_cap / C));
    struct Round {
        uint64_t w0, w1, a, len;
        bool continues;
        int si;
        uint32_t m;
        uint64_t ticket, bytes;
        uint32_t flags;          // VX_ROUND_* (the round timeline)
        uint64_t t_submit = 0;   // its reads queued (steady-clock ns)
    };
    std::vector<Round> rounds;
    for (uint64_t w0 = first; w0 < end; w0 += W) {
        const uint64_t w1 = std::min<uint64_t>(end, w0 + W);
        const uint64_t wmax = w1 == n ? std::max<uint64_t>(pl, last_len) : pl;
        const int ramp = (int)c->cfg.verify_ramp;
        const auto sched = chunk_schedule(wmax, C, w0 == first ? ramp : 0, w1 == end ? ramp : 0);
        for (size_t k = 0; k < sched.size(); ++k) {
            const uint64_t a = sched[k].first, len = sched[k].second;
            const uint32_t fl = (k == 0 ? VX_ROUND_NEW_WINDOW : 0u) |
                                (len < C && a < C && w0 == first ? VX_ROUND_HEAD_RAMP : 0u) |
                                (len < C && a >= C && w1 == end ? VX_ROUND_TAIL_RAMP : 0u);
            rounds.push_back(Round{w0, w1, a, len, k > 0, -1, 0, 0, 0, fl});
        }
    }
    const size_t nslots = c->slots.size();
    const size_t depth = nslots > 1 ? std::min<size_t>(kReadahead, nslots - 1) : 0;
    std::vector<std::vector<vx_files::ReadItem>> items(nslots);
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a, clk::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    // Timing events around each round's data copy and after its kernel
    // (start, end, kernel end), kept on the context and reused
    // (vx_last_verify / vx_last_verify_rounds).  An anchor event recorded on
    // an idle stream now maps GPU times onto the host clock of the call.
    size_t timed = 0;
    std::vector<uint64_t> timed_bytes;
    std::vector<vx_verify_round> tl;  // the round timeline, one per enqueued round
    std::vector<long> tl_ev;          // timed-copy index of each timeline round, -1 when untimed
    bool anchored = false;
    uint64_t t_anchor = 0;
    if (c->anchor_ev || hipEventCreate(&c->anchor_ev) == hipSuccess) {
        anchored = hipEventRecord(c->anchor_ev, c->slots[0].stream) == hipSuccess;
        t_anchor = vx_files::Readers::now_ns();
    }
    auto rel_ms = [&](uint64_t t_ns) { return t_ns ? ((double)t_ns - (double)c->verify_t0_ns) * 1e-6 : 0.0; };
    auto t_last_enqueue = clk::now();
    auto consume = [&] { fv.consume(); };
    // Reserve a slot for round r and queue its reads; false when no slot is
    // free and `block` is not set.
    auto start_read = [&](Round& r, bool block) -> bool {
        int si = -1;
        if (block) {
            si = cp.free_slot(consume);
            if (si < 0) rc = si;
        } else {
            rc = cp.try_free_slot(&si, consume);
        }
        if (rc || si < 0) return false;
        Slot& s = c->slots[si];
        reset_fill(s);
        if ((rc = ensure_stage(c, s))) return false;
        // lanes 4 KiB apart: every stage destination can take an O_DIRECT read
        const uint64_t pitch = align_up(r.len, vx_files::DirectIo::kBlock);
        auto& it = items[si];
        it.clear();
        uint32_t m = 0;
        for (uint64_t i = r.w0; i < r.w1; ++i) {
            const uint64_t len_i = i == n - 1 ? last_len : pl;
            if (r.a >= len_i && !(r.a == 0 && len_i == 0)) continue;  // piece already finished
            const uint64_t clen = std::min<uint64_t>(r.len, len_i - r.a);
            it.push_back(vx_files::ReadItem{s.h_stage + (uint64_t)m * pitch, i, r.a, clen});
            s.h_offsets[m] = (uint64_t)m * pitch;
            s.h_lens[m] = (uint32_t)clen;
            s.h_pidx[m] = (uint32_t)(i - first);
            s.h_poff[m] = r.a;
            s.h_tlen[m] = len_i;
            ++m;
        }
        r.m = m;
        if (m == 0) return true;  // nothing to read or hash: the slot stays free
        s.state = Slot::FILLING;  // reserved until the round is enqueued
        s.bytes = r.bytes = (uint64_t)(m - 1) * pitch + s.h_lens[m - 1];
        r.si = si;
        r.t_submit = vx_files::Readers::now_ns();
        r.ticket = rd.submit(it);
        return true;
    };
    size_t nr = 0;  // next round to read
    for (size_t ne = 0; ne < rounds.size() && !rc; ++ne) {
        while (nr < rounds.size() && nr <= ne + depth && start_read(rounds[nr], nr == ne)) ++nr;
        if (rc) break;
        Round& r = rounds[ne];
        if (r.m == 0) continue;
        rd.wait(r.ticket);
        vx_verify_round vr{};
        vr.read_submit_ms = rel_ms(r.t_submit);
        vr.read_done_ms = rel_ms(rd.done_ns(r.ticket));
        vr.enqueue_ms = rel_ms(vx_files::Readers::now_ns());
        vr.bytes = r.bytes;
        vr.offset = r.a;
        vr.lanes = r.m;
        vr.flags = r.flags;
        long ev_k = -1;
        rc = cp.round(r.si, r.m, r.continues, false, [&](Slot& sl, hipStream_t st) {
            bool ev = true;
            while (ev && c->copy_ev.size() < 3 * timed + 3) {
                hipEvent_t e = nullptr;
                ev = hipEventCreate(&e) == hipSuccess;
                if (ev) c->copy_ev.push_back(e);
            }
            ev = ev && hipEventRecord(c->copy_ev[3 * timed], st) == hipSuccess;
            if (hipMemcpyAsync(sl.d_arena, sl.h_stage, sl.bytes, hipMemcpyHostToDevice, st) != hipSuccess)
                return fail(VX_EDEVICE, "vx_verify_files: chunk H2D failed");
            if (ev && hipEventRecord(c->copy_ev[3 * timed + 1], st) == hipSuccess) {  // timing is best effort
                timed_bytes.push_back(sl.bytes);
                cp.copy_end = c->copy_ev[3 * timed + 1];  // doubles as the round's `copied` (copy stream)
                ev_k = (long)timed++;
            }
            return 0;
        });
        // after the round's chunk kernel (cp.round enqueued it on the slot's stream)
        if (!rc && ev_k >= 0 && hipEventRecord(c->copy_ev[3 * ev_k + 2], c->slots[r.si].stream) != hipSuccess)
            ev_k = -1;
        tl.push_back(vr);
        tl_ev.push_back(ev_k);
        t_last_enqueue = clk::now();
    }
    rd.wait();  // error path: no read may still target a stage
    for (auto& sl : c->slots)  // rounds read but never launched (error path)
        if (sl.state == Slot::FILLING) {
            reset_fill(sl);
            sl.state = Slot::FREE;
        }
    rc = cp.finish(fv.matched_out, nullptr, rc, fv.bad.data());
    vx_verify_trace& vt = c->last_verify;
    vt.tail_ms = ms(t_last_enqueue, clk::now());
    if (!rc && timed) {  // finish() waited for every round: the copy events are complete
        float a = 0, b = 0, busy = 0;
        for (size_t k = 0; k < timed; ++k) {
            (void)hipEventElapsedTime(&a, c->copy_ev[0], c->copy_ev[3 * k]);
            (void)hipEventElapsedTime(&b, c->copy_ev[0], c->copy_ev[3 * k + 1]);
            busy += b - a;
            vt.copy_bytes += timed_bytes[k];
        }
        vt.copy_busy_ms = busy;
        vt.copy_span_ms = b;
        vt.rounds = (uint32_t)timed;
        // GPU times on the call's host clock, through the anchor
        const double base = anchored ? ((double)t_anchor - (double)c->verify_t0_ns) * 1e-6 : 0.0;
        for (size_t k = 0; k < tl.size() && anchored; ++k) {
            if (tl_ev[k] < 0) continue;
            float x = 0;
            const size_t e = 3 * (size_t)tl_ev[k];
            if (hipEventElapsedTime(&x, c->anchor_ev, c->copy_ev[e]) == hipSuccess) tl[k].copy_start_ms = base + x;
            if (hipEventElapsedTime(&x, c->anchor_ev, c->copy_ev[e + 1]) == hipSuccess) tl[k].copy_end_ms = base + x;
            if (hipEventElapsedTime(&x, c->anchor_ev, c->copy_ev[e + 2]) == hipSuccess) tl[k].kernel_end_ms = base + x;
        }
    }
    c->last_rounds = std::move(tl);
    if (!rc)
        for (uint64_t i = 0; i < cnt; ++i)
            if (fv.bad[i]) fv.matched_out[i] = 0;
    fv.done = cnt;
    return rc;
}

// The GPU's per-block chain time on the split kernels and the PCIe rate: the
// cost model's hardware figures (vx_plan_verify), and the
// split's cold-start guesses before it has measured its own.
constexpr double kChainBlock = 0.76e-6, kPcieRate = 52.0 * (1ull << 30);

// ---- the self-balancing split (vx_verify_files_split) ----
// The claim word: head (low 32 bits) | stop (high 32).  The pool moves head
// up one piece per compare-and-swap (vx_split_claim); the engine moves stop
// down by a group (split_take_tail).  Neither side can take a piece the other
// has, and a group the engine asks for is cut to what is still unclaimed.
// The claimed pieces are [returned, *was) (*was: the stop before the claim).
// expect: the stop this engine left (UINT64_MAX: any); a different stop means
// an engine the split was not declared for (vx_split.engines) claims from it,
// and the call returns UINT64_MAX.
uint64_t split_take_tail(vx_split* s, uint64_t k, uint64_t expect = UINT64_MAX, uint64_t* was = nullptr) {
    uint64_t w = __atomic_load_n(&s->word, __ATOMIC_ACQUIRE);
    for (;;) {
        const uint64_t head = w & 0xffffffffull, stop = w >> 32;
        if (was) *was = stop;
        if (expect != UINT64_MAX && stop != expect) return UINT64_MAX;
        const uint64_t take = std::min(k, stop > head ? stop - head : 0);
        if (take == 0) return stop;
        const uint64_t nw = head | ((stop - take) << 32);
        if (__atomic_compare_exchange_n(&s->word, &w, nw, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE))
            return stop - take;
    }
}

// Streaming chunk rounds over pieces the engine claims from the top of the
// split as it goes.  A claimed piece takes a lane from its first chunk to its
// last, one C-byte chunk per round; every round carries all active lanes and
// the group that joins it (batch_chunked_gather's streaming rounds, here with
// the group sized at run time).  Before forming a round the engine estimates
//   T_engine(j) = the rounds its lanes (and j new pieces) still need, each
//                 max(bytes / intake, longest chunk's chain), plus the first
//                 round's read and the last kernel's chain
//   T_pool(j)   = (unclaimed - engines x j + half the pool's pieces in hand)
//                 / the pool's pace
// and takes the largest j with T_engine(j) <= T_pool(j).  The rates are
// measured in this call — the intake from the GPU copy events (first copy
// start to last copy end), the chain per 64-byte block from the kernel
// events, the pool's pace over its last 4 ms of vx_split_done — except for
// the first group, which starts from earlier split calls on this context (or
// the caller's per-thread rate, the PCIe rate and kChainBlock); its T_engine
// adds the lag earlier calls' single groups ended behind their prediction
// (the readers' start-up and the kernels trailing the copies).  No later
// group is formed until both sides have rates, and one only if it rides the
// active lanes' rounds and shortens the predicted end by a tenth — except
// for pieces of one chunk, whose groups cost one round each: those keep the
// first group's rule until the rates are in, and then only the model's.  Alone on
// the split (engines 1) the engine's pieces are the contiguous tail
// [*lowest, end); beside other engines, the groups it took.
int verify_split(FileVerify& fv, vx_files::Readers& rd, vx_split* sp, uint64_t n, uint32_t pl, uint64_t total,
                 uint64_t C, uint64_t* lowest, int regime) {
    vx_ctx* c = fv.c;
    const uint64_t first = sp->first, end = sp->end, cnt = end - first;
    const uint64_t last_len = total - (n - 1) * (uint64_t)pl;
    auto plen = [&](uint64_t i) { return i == n - 1 ? last_len : (uint64_t)pl; };
    ChunkPipe cp(c);
    c->last_split.clear();
    int rc = cp.open(cnt, fv.expected + 20 * first, "vx_verify_files_split");
    if (!rc && c->verify_copy_stream) rc = cp.use_copy_stream();
    const uint64_t longest = std::max<uint64_t>(pl, last_len);
    const uint64_t pitch = align_up(std::min<uint64_t>(C, longest), vx_files::DirectIo::kBlock);
    const Slot& s0 = c->slots[0];
    uint64_t max_lanes = std::max<uint64_t>(1, std::min<uint64_t>(s0.cap, s0.arena_cap / pitch));
    *lowest = end;

    struct Lane {
        uint64_t piece, a;
        bool ramp;  // joined in the first round: chunks C/4, C/4, C/2, then C
    };
    std::vector<Lane> act;  // claimed pieces with chunks left, in join order
    // verify_chunked's ramps (chunk_schedule, depth 1), per lane.  Head: the
    // first group's first round is a C/4 chain and a quarter of the bytes, so
    // the call's first read and the copy that nothing overlaps are short
    // (later groups join rounds whose chain is C anyway).  Tail, every lane:
    // its last C bytes go as C/2, C/4, rest, so the chain left after the
    // call's last copy is C/4's, not C's.
    const bool ramp_ok = C >= 4 * vx_files::DirectIo::kBlock;
    auto chunk_len = [&](uint64_t L, uint64_t a, bool head) {
        if (!ramp_ok || L < 2 * C) return std::min<uint64_t>(C, L - a);
        const uint64_t q = C / 4, tail_from = (L - C + q - 1) / q * q;
        if (head && a < C) return a < C / 2 ? q : C / 2;
        if (a < tail_from) return std::min<uint64_t>(C, tail_from - a);
        const uint64_t off = a - tail_from;
        return off == 0 ? std::min<uint64_t>(C / 2, L - a) : off == C / 2 ? std::min<uint64_t>(q, L - a) : L - a;
    };
    // chunk lengths of a full-length piece joining now (ramped or not)
    auto schedule = [&](bool ramp) {
        std::vector<uint64_t> v;
        for (uint64_t a = 0; a < pl;) v.push_back(chunk_len(pl, a, ramp)), a += v.back();
        if (v.empty()) v.push_back(0);
        return v;
    };
    const std::vector<uint64_t> sched_plain = schedule(false), sched_ramp = schedule(true);
    const bool one_round = c->split_one_round && sched_plain.size() == 1;  // every piece is one chunk (pl <= C)
    // One-chunk pieces' rounds are whole groups: a smaller round starts the
    // first copy sooner and ends the last kernel sooner (64 KiB pieces: 256 ->
    // 64 MiB rounds, 50.5-52.5 -> 55.9-56.0 GiB/s; tools/split_rules_ab.py),
    // but not below 1,024 lanes, whose kernels run one piece's chain each.
    if (one_round && c->split_round_cap)
        max_lanes = std::min(max_lanes, std::max<uint64_t>(1024, c->split_round_cap / pitch));
    struct Round {
        int si = -1;
        uint32_t m = 0;
        bool continues = false;
        uint64_t ticket = 0, bytes = 0, max_chunk = 0, t_submit = 0;
    };
    std::deque<Round> formed;  // reads queued, not yet enqueued
    const size_t nslots = c->slots.size();
    const size_t depth = nslots > 1 ? std::min<size_t>(kReadahead, nslots - 1) : 0;
    std::vector<std::vector<vx_files::ReadItem>> items(nslots);
    using clk = std::chrono::steady_clock;
    // enqueued rounds: bytes, longest chunk, timing-event index (-1: untimed)
    struct Sent {
        uint64_t bytes, max_chunk;
        long ev;
        bool continues;
    };
    std::vector<Sent> sent;
    size_t timed = 0, measured_upto = 0;  // rounds [0, measured_upto) are in the rates below
    // The copy intake so far: bytes copied over first copy start -> last copy
    // end (a copy that waited for its reads counts the wait).
    double in_bytes = 0, in_ms = 0, in_n = 0;
    float first_cs = -1;
    // every measured copy: (end ms, bytes, longest chunk), for the steady-state
    // intake the next call starts from
    struct CopyEnd {
        double end_ms;
        uint64_t bytes, max_chunk;
    };
    std::vector<CopyEnd> copy_ends;
    std::vector<double> block_ns;         // measured chain per 64-byte block, one per round
    std::vector<uint64_t> timed_bytes;
    std::vector<vx_verify_round> tl;
    std::vector<long> tl_ev;
    bool anchored = false;
    uint64_t t_anchor = 0;
    if (c->anchor_ev || hipEventCreate(&c->anchor_ev) == hipSuccess) {
        anchored = hipEventRecord(c->anchor_ev, c->slots[0].stream) == hipSuccess;
        t_anchor = vx_files::Readers::now_ns();
    }
    auto rel_ms = [&](uint64_t t_ns) { return t_ns ? ((double)t_ns - (double)c->verify_t0_ns) * 1e-6 : 0.0; };
    auto consume = [&] { fv.consume(); };
    const double pool_threads = sp->cpu_threads;
    // engines claiming from this split at once (vx_split.engines): each takes
    // an equal share of what the pool does not
    const uint64_t engines = std::max<uint32_t>(1, sp->engines);
    std::vector<std::pair<uint64_t, uint64_t>> mine;  // this engine's claims, [lo, hi), in claim order
    std::vector<std::pair<uint64_t, uint64_t>> pool_samples;  // (steady ns, pool_done) at each decision
    constexpr uint64_t kPoolWindowNs = 4000000;              // the pool's pace: its last 4 ms
    const double thread_rate0 = c->split_pool_thread_rate[regime].any() ? c->split_pool_thread_rate[regime].get(c->split_learn)
                                : sp->cpu_thread_rate > 0    ? sp->cpu_thread_rate
                                                             : 2.2e9;
    const double pool_rate0 = pool_threads * thread_rate0 / (double)pl;
    double last_p = 0;  // the pool's pace at the last decision
    // the first group's predicted ends (call clock, ms; the engine's without
    // the learned lag) and the engine's span, and whether any later group
    // joined: the lag's sample
    double first_end_ms = -1, first_pool_end_ms = -1, first_span_ms = 0, lag_used = 0;
    bool later_group = false;

    // Fold newly finished rounds into the copy and chain rates (events are
    // queried, never waited for).
    size_t copied_upto = 0;  // rounds whose copy is in the intake above
    auto measure = [&] {
        // copies as soon as they end (the first rate arrives a kernel earlier)
        while (copied_upto < sent.size()) {
            const Sent& r = sent[copied_upto];
            if (r.ev >= 0) {
                const size_t e = 3 * (size_t)r.ev;
                if (hipEventQuery(c->copy_ev[e + 1]) != hipSuccess) break;
                float cs = 0, ce = 0;
                if (hipEventElapsedTime(&cs, c->copy_ev[0], c->copy_ev[e]) == hipSuccess &&
                    hipEventElapsedTime(&ce, c->copy_ev[0], c->copy_ev[e + 1]) == hipSuccess) {
                    if (first_cs < 0) first_cs = cs;
                    in_bytes += (double)r.bytes;
                    in_ms = (double)ce - (double)first_cs;
                    in_n += 1;
                    copy_ends.push_back(CopyEnd{(double)ce, r.bytes, r.max_chunk});
                }
            }
            ++copied_upto;
        }
        // kernels: the chain per block, and which rounds are done
        while (measured_upto < sent.size()) {
            const Sent& r = sent[measured_upto];
            if (r.ev < 0) {
                ++measured_upto;
                continue;
            }
            const size_t e = 3 * (size_t)r.ev;
            if (hipEventQuery(c->copy_ev[e + 2]) != hipSuccess) break;  // kernel not done yet
            float k0 = 0, k1 = 0, ce = 0;
            // the kernel starts after its copy and, when its lanes continue, after
            // the previous round's kernel
            long prev = -1;
            for (size_t k = measured_upto; r.continues && k-- > 0;)
                if (sent[k].ev >= 0) {
                    prev = sent[k].ev;
                    break;
                }
            if (hipEventElapsedTime(&ce, c->copy_ev[0], c->copy_ev[e + 1]) == hipSuccess &&
                hipEventElapsedTime(&k1, c->copy_ev[0], c->copy_ev[e + 2]) == hipSuccess) {
                if (prev >= 0) (void)hipEventElapsedTime(&k0, c->copy_ev[0], c->copy_ev[3 * (size_t)prev + 2]);
                const double kern_ms = (double)k1 - std::max<double>(ce, prev >= 0 ? k0 : 0.0);
                const double blocks = (double)((r.max_chunk + 63) / 64);
                if (kern_ms > 0 && blocks > 0) block_ns.push_back(kern_ms * 1e6 / blocks);
            }
            ++measured_upto;
        }
    };
    // How many pieces to take now (0..room).
    // mode 0: a round after the first (no group until both sides have rates);
    // 1: the first round (the cold-start answer); 2: nothing is in flight and
    // the rates are not all in: decide with what there is.
    auto decide = [&](uint64_t room, int mode, bool* measured) -> uint64_t {
        measure();
        const uint64_t w = __atomic_load_n(&sp->word, __ATOMIC_ACQUIRE);
        const uint64_t head = w & 0xffffffffull, stop = w >> 32;
        const uint64_t unclaimed = stop > head ? stop - head : 0;
        if (unclaimed == 0 || room == 0) return 0;
        const uint64_t done = __atomic_load_n(&sp->pool_done, __ATOMIC_ACQUIRE);
        const uint64_t now = vx_files::Readers::now_ns();
        const double el = ((double)now - (double)sp->start_ns) * 1e-9;
        const bool pool_measured = pool_threads == 0 || (done >= std::max(4.0, pool_threads) && el > 0);
        // The pool's rate over the last few ms (its start-up — threads
        // spawning, first pieces — is not its pace), or since the start.
        double p = pool_threads == 0 ? 0.0 : pool_measured ? (double)done / el : pool_rate0;
        bool windowed = pool_threads == 0;
        for (size_t k = pool_samples.size(); pool_measured && pool_threads > 0 && k-- > 0;) {
            const auto& sm = pool_samples[k];
            if (now - sm.first >= kPoolWindowNs) {
                if (done > sm.second) p = (double)(done - sm.second) / ((double)(now - sm.first) * 1e-9);
                windowed = done > sm.second;
                break;
            }
        }
        pool_samples.emplace_back(now, done);
        // A later group needs the pool's pace over a window (not its start-up)
        // and the engine's intake over two copies.
        *measured = in_n >= 2 && windowed;
        // The first group is decided before the pool has a pace: a rate since
        // the start is mostly its start-up, so it never goes below the rate the
        // caller measured alone (an over-claim cannot be handed back; an
        // under-claim is topped up once the rates are in).  Pieces that fit one
        // round (a group costs one round, not a piece's whole chain) keep
        // deciding so until the rates are in, rather than draining the pipeline.
        const bool cold = mode == 1 || (mode == 0 && one_round && !*measured);
        if (cold && pool_threads > 0) p = std::max(p, pool_rate0);
        // With the engine idle (mode 2), a pool that has finished nothing for
        // two of its piece times (at least the window) while pieces are still
        // unclaimed is held up — vortex's rayon pool also hashes downloads —
        // so it counts as stopped and the engine takes what it can, instead
        // of leaving the rest to it.
        if (mode == 2 && pool_threads > 0 && unclaimed > 0) {
            const uint64_t win = std::max<uint64_t>(kPoolWindowNs, (uint64_t)(2e9 * (double)pl / thread_rate0));
            for (size_t k = pool_samples.size() - 1; k-- > 0;)  // (the last sample is this call's)
                if (now - pool_samples[k].first >= win) {
                    if (pool_samples[k].second == done) p = 0;
                    break;
                }
        }
        // pieces the pool holds count half done
        const double in_hand = 0.5 * ((double)(head - first) - (double)std::min<uint64_t>(done, head - first));
        // The engine's chain per block is a property of the kernel, known within
        // a few % before any round of this call ends (kChainBlock); waiting for
        // a kernel end put the first measured group a whole round later.
        if (!*measured && !cold && mode == 0) return 0;
        if (windowed) last_p = p;
        const double rin = in_n >= 2 && in_ms > 0 ? in_bytes / (in_ms * 1e-3)
                           : c->split_rin[regime].any() ? (c->split_learn ? c->split_rin[regime].top() : c->split_rin[regime].get(0))
                                                  : kPcieRate;
        double bns = c->split_bns[regime].any() ? c->split_bns[regime].get(c->split_learn) : kChainBlock * 1e9;
        if (!block_ns.empty()) {
            std::vector<double> b = block_ns;
            std::nth_element(b.begin(), b.begin() + b.size() / 2, b.end());
            bns = b[b.size() / 2];
        }
        auto round_s = [&](double bytes, uint64_t chunk) {
            return std::max(bytes / rin, (double)((chunk + 63) / 64) * bns * 1e-9);
        };
        // rounds queued ahead of the new group (enqueued and not finished, or
        // formed), in order; nothing sent yet: the first round's read too
        double t_queued = 0;
        uint64_t last_k = 0;  // the longest chunk of the last round queued
        for (size_t k = measured_upto; k < sent.size(); ++k)
            t_queued += round_s((double)sent[k].bytes, sent[k].max_chunk), last_k = sent[k].max_chunk;
        for (const Round& r : formed) t_queued += round_s((double)r.bytes, r.max_chunk), last_k = r.max_chunk;
        // future rounds of the active lanes: bytes per round index
        std::vector<double> fut;
        std::vector<uint64_t> fut_max;  // each future round's longest chunk
        for (const Lane& l : act) {
            const uint64_t L = plen(l.piece);
            uint64_t a = l.a;
            for (size_t r = 0; a < L; ++r) {
                const uint64_t k = chunk_len(L, a, l.ramp);
                if (fut.size() <= r) fut.resize(r + 1, 0.0), fut_max.resize(r + 1, 0);
                fut[r] += (double)k;
                fut_max[r] = std::max(fut_max[r], k);
                a += k;
            }
        }
        const std::vector<uint64_t>& js = mode == 1 ? sched_ramp : sched_plain;
        // (the lag from three calls on: the median of one or two is their noise)
        lag_used = mode == 1 && c->split_lag_on && c->split_lag[regime].n >= 3 ? c->split_lag[regime].get(c->split_learn) : 0.0;
        // Each round costs max(its bytes over the intake, its chain), copies
        // overlapping the previous round's kernel; after the last copy, the
        // last kernel's chain; before the first, the first round's read.
        const bool first_read = sent.empty() && formed.empty();
        auto t_engine = [&](uint64_t j) {
            double t = t_queued;
            uint64_t k_end = last_k;
            const size_t R = std::max<size_t>(fut.size(), j ? js.size() : 0);
            for (size_t r = 0; r < R; ++r) {
                double b = r < fut.size() ? fut[r] : 0.0;
                uint64_t k = r < fut_max.size() ? fut_max[r] : 0;
                if (j && r < js.size()) b += (double)j * (double)js[r], k = std::max(k, js[r]);
                if (b > 0) t += round_s(b, k) + (r == 0 && first_read ? b / rin : 0.0), k_end = k;
            }
            return t + (double)((k_end + 63) / 64) * bns * 1e-9 + lag_used;
        };
        auto t_pool = [&](uint64_t j) {  // the others take an equal share each
            const double left = (double)unclaimed - (double)(engines * j);
            return p > 0 ? (std::max(0.0, left) + in_hand) / p : std::numeric_limits<double>::infinity();
        };
        // A later group rides the rounds the active lanes still have; one that
        // needs more than one round beyond them adds a tail of rounds that are
        // one chain each with PCIe idle, which a rate misread from a short
        // window (a host-wide stall slows both sides for 10+ ms) cannot repay.
        if (mode == 0 && !act.empty() && js.size() > fut.size() + 1) return 0;
        // the largest j in [0, min(unclaimed, room)] with t_engine(j) <= t_pool(j):
        // t_engine grows with j and t_pool shrinks, so bisect
        auto ok = [&](uint64_t j) { return t_engine(j) <= t_pool(j); };
        uint64_t lo = 0, hi = std::min(engines == 1 ? unclaimed : (unclaimed + engines - 1) / engines, room);
        if (ok(hi)) {
            lo = hi;
        } else if (ok(1)) {
            lo = 1;
            while (lo + 1 < hi) {
                const uint64_t mid = lo + (hi - lo) / 2;
                (ok(mid) ? lo : hi) = mid;
            }
        }

        // and a later group must shorten the predicted end by a tenth (a group
        // of one-round pieces risks one round, and is a small share of the end)
        if (mode == 0 && !one_round && lo > 0 &&
            std::max(t_engine(lo), t_pool(lo)) > 0.9 * std::max(t_engine(0), t_pool(0)))
            lo = 0;
        c->last_split.push_back(vx_ctx::SplitDecision{
            ((double)vx_files::Readers::now_ns() - (double)c->verify_t0_ns) * 1e-6, p, rin, bns,
            t_engine(lo) * 1e3, t_pool(lo) * 1e3, unclaimed, lo, (uint64_t)act.size(), done, (uint32_t)mode,
            *measured ? 1u : 0u, lag_used * 1e3});
        return lo;
    };

    // Form the next round into a slot: the active lanes' next chunks plus a
    // group claimed now.  1 = formed, 0 = nothing left for the engine,
    // -1 = no slot free (block = false) or an error (rc set).
    bool formed_any = false;
    auto form = [&](bool block) -> int {
        int si = -1;
        for (int attempt = 0;; ++attempt) {
            if (block) {
                si = cp.free_slot(consume);
                if (si < 0) {
                    rc = si;
                    return -1;
                }
            } else {
                if ((rc = cp.try_free_slot(&si, consume))) return -1;
                if (si < 0) return -1;
            }
            bool measured = false;
            bool inflight = false;
            for (const Slot& q : c->slots) inflight |= q.state == Slot::INFLIGHT;
            const int mode = !formed_any && attempt == 0 ? 1 : (block && !inflight && formed.empty()) ? 2 : 0;
            const uint64_t j = decide(max_lanes - std::min<uint64_t>(max_lanes, act.size()), mode, &measured);
            if (j > 0 || !act.empty()) {
                Slot& s = c->slots[si];
                reset_fill(s);
                if ((rc = ensure_stage(c, s))) return -1;
                auto& it = items[si];
                it.clear();
                // the round's lanes: the active ones, then the group claimed now
                std::vector<Lane> lanes = act;
                const bool continues = !act.empty();
                if (j) {
                    // alone on the split, the stop is where this engine left it
                    uint64_t old = 0;
                    const uint64_t lo = split_take_tail(sp, j, engines == 1 ? *lowest : UINT64_MAX, &old);
                    if (lo == UINT64_MAX) {
                        rc = fail(VX_EINVAL, "vx_verify_files_split: another engine claims from this split");
                        return -1;
                    }
                    if (lo < old && !mine.empty() && mine.back().first == old)
                        mine.back().first = lo;  // right below the last group: one range (one D2H)
                    else if (lo < old)
                        mine.emplace_back(lo, old);
                    for (uint64_t i = lo; i < old; ++i) lanes.push_back(Lane{i, 0, !formed_any});
                    *lowest = std::min(*lowest, lo);
                    const vx_ctx::SplitDecision& d = c->last_split.back();
                    if (mode == 1) {
                        first_span_ms = d.t_engine_ms - lag_used * 1e3;
                        first_end_ms = d.t_ms + first_span_ms;
                        first_pool_end_ms = d.t_ms + d.t_pool_ms;
                    } else if (lo < old) {
                        later_group = true;
                    }
                }
                // lanes sit one round pitch apart: the round's longest chunk,
                // 4 KiB aligned for O_DIRECT (ramp rounds copy no gaps)
                uint64_t max_chunk = 0;
                for (const Lane& l : lanes) max_chunk = std::max(max_chunk, chunk_len(plen(l.piece), l.a, l.ramp));
                const uint64_t rp = std::max<uint64_t>(vx_files::DirectIo::kBlock,
                                                       align_up(max_chunk, vx_files::DirectIo::kBlock));
                uint32_t m = 0;
                std::vector<Lane> keep;
                // one-chunk pieces are whole pieces in increasing order: runs of
                // them inside one file go out as one pread (as in verify_whole)
                vx_files::Runs runs = rd.runs(one_round && c->split_one_round != 2 ? 4ull << 20 : 0);
                for (const Lane& l : lanes) {
                    const uint64_t L = plen(l.piece), clen = chunk_len(L, l.a, l.ramp);
                    if (one_round)
                        runs.add(it, s.h_stage + (uint64_t)m * rp, l.piece, clen);
                    else
                        it.push_back(vx_files::ReadItem{s.h_stage + (uint64_t)m * rp, l.piece, l.a, clen});
                    s.h_offsets[m] = (uint64_t)m * rp;
                    s.h_lens[m] = (uint32_t)clen;
                    s.h_pidx[m] = (uint32_t)(l.piece - first);
                    s.h_poff[m] = l.a;
                    s.h_tlen[m] = L;
                    ++m;
                    if (l.a + clen < L) keep.push_back(Lane{l.piece, l.a + clen, l.ramp});
                }
                act.swap(keep);
                if (m == 0) continue;  // the group came back empty (the pool took the rest)
                formed_any = true;
                s.state = Slot::FILLING;  // reserved until the round is enqueued
                Round r;
                r.si = si;
                r.m = m;
                r.continues = continues;
                r.bytes = s.bytes = (uint64_t)(m - 1) * rp + s.h_lens[m - 1];
                r.max_chunk = max_chunk;
                r.t_submit = vx_files::Readers::now_ns();
                r.ticket = rd.submit(it);
                formed.push_back(r);
                return 1;
            }
            // Nothing to form.  While the rates are not all in, wait for a round
            // in flight and decide again (mode 2 once none is left); with
            // them, the engine is done: the pool takes the rest.
            if (!block || measured || mode == 2) return 0;
            if (inflight) {
                if ((rc = reap(c, true))) return -1;
                consume();
            }
        }
    };

    auto t_last_enqueue = clk::now();
    for (;;) {
        while (formed.size() <= depth) {
            const int f = form(formed.empty());
            if (f <= 0) break;
        }
        if (rc || formed.empty()) break;
        Round r = formed.front();
        formed.pop_front();
        rd.wait(r.ticket);
        vx_verify_round vr{};
        vr.read_submit_ms = rel_ms(r.t_submit);
        vr.read_done_ms = rel_ms(rd.done_ns(r.ticket));
        vr.enqueue_ms = rel_ms(vx_files::Readers::now_ns());
        vr.bytes = r.bytes;
        vr.lanes = r.m;
        vr.flags = r.continues ? 0u : VX_ROUND_NEW_WINDOW;
        long ev_k = -1;
        rc = cp.round(r.si, r.m, r.continues, false, [&](Slot& sl, hipStream_t st) {
            bool ev = true;
            while (ev && c->copy_ev.size() < 3 * timed + 3) {
                hipEvent_t e = nullptr;
                ev = hipEventCreate(&e) == hipSuccess;
                if (ev) c->copy_ev.push_back(e);
            }
            ev = ev && hipEventRecord(c->copy_ev[3 * timed], st) == hipSuccess;
            if (hipMemcpyAsync(sl.d_arena, sl.h_stage, sl.bytes, hipMemcpyHostToDevice, st) != hipSuccess)
                return fail(VX_EDEVICE, "vx_verify_files_split: chunk H2D failed");
            if (ev && hipEventRecord(c->copy_ev[3 * timed + 1], st) == hipSuccess) {
                timed_bytes.push_back(sl.bytes);
                cp.copy_end = c->copy_ev[3 * timed + 1];
                ev_k = (long)timed++;
            }
            return 0;
        });
        if (!rc && ev_k >= 0 && hipEventRecord(c->copy_ev[3 * ev_k + 2], c->slots[r.si].stream) != hipSuccess)
            ev_k = -1;
        sent.push_back(Sent{r.bytes, r.max_chunk, ev_k, r.continues});
        tl.push_back(vr);
        tl_ev.push_back(ev_k);
        t_last_enqueue = clk::now();
        if (rc) break;
    }
    rd.wait();  // error path: no read may still target a stage
    for (auto& sl : c->slots)
        if (sl.state == Slot::FILLING) {
            reset_fill(sl);
            sl.state = Slot::FREE;
        }
    // rows of this engine's pieces, relative to first
    std::vector<std::pair<uint64_t, uint64_t>> rows;
    for (const auto& r : mine) {
        rows.emplace_back(r.first - first, r.second - first);
        for (uint64_t i = r.first; i < r.second; ++i) cp.bytes += plen(i);
    }
    rc = cp.finish_rows(fv.matched_out, rc, fv.bad.data(), rows);
    vx_verify_trace& vt = c->last_verify;
    vt.tail_ms = std::chrono::duration<double, std::milli>(clk::now() - t_last_enqueue).count();
    if (!rc && timed) {
        float a = 0, b = 0, busy = 0;
        for (size_t k = 0; k < timed; ++k) {
            (void)hipEventElapsedTime(&a, c->copy_ev[0], c->copy_ev[3 * k]);
            (void)hipEventElapsedTime(&b, c->copy_ev[0], c->copy_ev[3 * k + 1]);
            busy += b - a;
            vt.copy_bytes += timed_bytes[k];
        }
        vt.copy_busy_ms = busy;
        vt.copy_span_ms = b;
        vt.rounds = (uint32_t)timed;
        const double base = anchored ? ((double)t_anchor - (double)c->verify_t0_ns) * 1e-6 : 0.0;
        for (size_t k = 0; k < tl.size() && anchored; ++k) {
            if (tl_ev[k] < 0) continue;
            float x = 0;
            const size_t e = 3 * (size_t)tl_ev[k];
            if (hipEventElapsedTime(&x, c->anchor_ev, c->copy_ev[e]) == hipSuccess) tl[k].copy_start_ms = base + x;
            if (hipEventElapsedTime(&x, c->anchor_ev, c->copy_ev[e + 1]) == hipSuccess) tl[k].copy_end_ms = base + x;
            if (hipEventElapsedTime(&x, c->anchor_ev, c->copy_ev[e + 2]) == hipSuccess) tl[k].kernel_end_ms = base + x;
        }
    }
    c->last_rounds = std::move(tl);
    if (!rc) {
        for (const auto& r : rows)
            for (uint64_t i = r.first; i < r.second; ++i)
                if (fv.bad[i]) fv.matched_out[i] = 0;
        // the next split call's cold start (this host, this load): this
        // call's figures join the last calls' (Learned)
        measure();
        // the steady-state intake: the full-chunk rounds' bytes over the time
        // from the copy before the first of them to the last one's end (the
        // ramps' short rounds and the chain-bound tail would understate it,
        // and the next call would claim too little)
        {
            size_t a = copy_ends.size(), b = 0;
            for (size_t k = 0; k < copy_ends.size(); ++k)
                if (copy_ends[k].max_chunk >= C) a = std::min(a, k), b = k;
            double bytes = 0;
            for (size_t k = a + 1; k <= b && a < copy_ends.size(); ++k) bytes += (double)copy_ends[k].bytes;
            const double ms = a < b ? copy_ends[b].end_ms - copy_ends[a].end_ms : 0.0;
            if (ms > 0 && bytes > 0) c->split_rin[regime].add(bytes / (ms * 1e-3));
        }
        if (!block_ns.empty()) {
            std::nth_element(block_ns.begin(), block_ns.begin() + block_ns.size() / 2, block_ns.end());
            c->split_bns[regime].add(block_ns[block_ns.size() / 2]);
        }
        if (last_p > 0 && pool_threads > 0) c->split_pool_thread_rate[regime].add(last_p * (double)pl / pool_threads);
        // The lag: how much later than predicted the engine's last kernel
        // ended, less how much later than predicted the pool's last verdict
        // came (vx_split.pool_last_ns), both against the first group's
        // decision.
        double end_ms = -1;
        for (const auto& r : c->last_rounds) end_ms = std::max(end_ms, r.kernel_end_ms);
        if (anchored && !later_group && engines == 1 && first_end_ms > 0 && end_ms > 0 && first_span_ms > 0) {
            double err = end_ms - first_end_ms;
            bool ok = true;
            if (pool_threads > 0) {
                // A pool still verifying its last pieces is waited for (polled,
                // at most 3x their estimated time + 50 ms): estimating its end
                // instead would miss the stalls that come after the engine's,
                // while counting those before it, and bias the lag up.  A pool
                // that has reported nothing is not waited for.
                uint64_t head = 0, stop = 0, done = 0, last_ns = 0;
                auto load = [&] {
                    const uint64_t w = __atomic_load_n(&sp->word, __ATOMIC_ACQUIRE);
                    head = w & 0xffffffffull, stop = w >> 32;
                    done = __atomic_load_n(&sp->pool_done, __ATOMIC_ACQUIRE);
                    last_ns = __atomic_load_n(&sp->pool_last_ns, __ATOMIC_ACQUIRE);
                };
                auto busy = [&] { return stop > head || done < head - first; };
                load();
                if (busy() && done > 0 && last_p > 0) {
                    const double left = 0.5 * (double)(head - first - std::min(done, head - first)) +
                                        (double)(stop > head ? stop - head : 0);
                    const uint64_t until = vx_files::Readers::now_ns() + (uint64_t)((3.0 * left / last_p + 0.05) * 1e9);
                    while (busy() && vx_files::Readers::now_ns() < until) {
                        std::this_thread::sleep_for(std::chrono::microseconds(200));
                        load();
                    }
                }
                ok = !busy() && last_ns && first_pool_end_ms > 0;
                if (ok) err -= ((double)last_ns - (double)c->verify_t0_ns) * 1e-6 - first_pool_end_ms;
            }
            if (ok) {
                const double v = std::clamp(err, -0.25 * first_span_ms, 0.5 * first_span_ms) * 1e-3;
                c->split_lag[regime].add(v);
            }
        }
    }
    fv.done = 0;
    for (const auto& r : rows) fv.done += r.second - r.first;
    return rc;
}

// Strided host batches of long pieces: every piece inside
// one registered range at a constant host stride, all of one length except
// possibly a shorter last piece — a bulk verify over a contiguous host copy
// of the torrent (torrent.rs:724-740), or the bench's e2e sample.  Round k of
// a window moves bytes [k*C, (k+1)*C) of each of its pieces with ONE
// hipMemcpy2DAsync (source pitch = host stride; 53 GiB/s like a flat copy,
// profiles/r01/h2d/h2d2d.json), and the chunk kernel continues each piece's
// state.  So the transfer is back to back and only the last round's short
// chain trails it, instead of a whole-piece chain per slot.
bool strided_batch(const vx_ctx* c, const uint8_t* const* ptrs, const uint32_t* lens, size_t n,
                   uint64_t* host_stride) {
    const uint64_t C = c->cfg.batch_chunk;
    if (n == 0 || C == 0 || c->slots[0].arena_cap < C) return false;
    const uint32_t L = lens[0];
    if (L < 2 * C || L > c->cfg.max_piece_len || lens[n - 1] == 0 || lens[n - 1] > L) return false;
    const uintptr_t p0 = reinterpret_cast<uintptr_t>(ptrs[0]);
    const uintptr_t hs = n > 1 ? reinterpret_cast<uintptr_t>(ptrs[1]) - p0 : L;
    if (hs < L || hs > (1ull << 40)) return false;
    for (size_t i = 0; i + 1 < n; ++i)
        if (lens[i] != L || reinterpret_cast<uintptr_t>(ptrs[i]) != p0 + i * hs) return false;
    if (reinterpret_cast<uintptr_t>(ptrs[n - 1]) != p0 + (n - 1) * hs) return false;
    if (!is_registered(c, ptrs[0], (n - 1) * hs + lens[n - 1])) return false;
    *host_stride = hs;
    return true;
}

int batch_chunked(vx_ctx* c, const uint8_t* const* ptrs, const uint32_t* lens, const uint8_t* expected, size_t n,
                  uint8_t* matched_out, uint8_t* digests_out, uint64_t hs) {
    const uint64_t C = c->cfg.batch_chunk;
    const uint64_t L = lens[0], Llast = lens[n - 1];
    const uint8_t* base = ptrs[0];
    ChunkPipe cp(c);
    int rc = cp.open(n, expected, "batch");
    for (size_t i = 0; i < n; ++i) cp.bytes += lens[i];
    const Slot& s0 = c->slots[0];
    const uint64_t W = std::max<uint64_t>(1, std::min<uint64_t>(s0.cap, s0.arena_cap / C));
    const uint64_t rounds = (L + C - 1) / C;
    for (uint64_t w0 = 0; w0 < n && !rc; w0 += W) {
        const uint64_t w1 = std::min<uint64_t>(n, w0 + W);
        const bool short_last = w1 == n && Llast != L;
        const uint64_t full_rows = (w1 - w0) - (short_last ? 1 : 0);
        for (uint64_t k = 0; k < rounds && !rc; ++k) {
            const uint64_t a = k * C;
            const uint64_t width = std::min<uint64_t>(C, L - a);   // every full-length row
            const uint64_t dpitch = align_up(width, kAlign);       // <= C
            const uint64_t last_w = short_last && a < Llast ? std::min<uint64_t>(C, Llast - a) : 0;
            const uint32_t m = (uint32_t)(full_rows + (last_w ? 1 : 0));
            if (m == 0) continue;
            const int si = cp.free_slot([] {});
            if (si < 0) {
                rc = si;
                break;
            }
            Slot& s = c->slots[si];
            reset_fill(s);
            for (uint32_t r = 0; r < m; ++r) {
                const bool is_last = r == full_rows;
                s.h_offsets[r] = (uint64_t)r * dpitch;
                s.h_lens[r] = (uint32_t)(is_last ? last_w : width);
                s.h_pidx[r] = (uint32_t)(is_last ? n - 1 : w0 + r);
                s.h_poff[r] = a;
                s.h_tlen[r] = is_last ? Llast : L;
            }
            rc = cp.round(si, m, k > 0, false, [&](Slot& sl, hipStream_t st) {
                if (full_rows && hipMemcpy2DAsync(sl.d_arena, dpitch, base + w0 * hs + a, hs, width, full_rows,
                                                  hipMemcpyHostToDevice, st) != hipSuccess)
                    return fail(VX_EDEVICE, "batch: chunk 2D H2D failed");
                if (last_w && hipMemcpyAsync(sl.d_arena + full_rows * dpitch, ptrs[n - 1] + a, last_w,
                                             hipMemcpyHostToDevice, st) != hipSuccess)
                    return fail(VX_EDEVICE, "batch: chunk H2D failed");
                return 0;
            });
        }
        cp.end_window();
    }
    return cp.finish(matched_out, digests_out, rc);
}
// Registered host batches that are not strided: pieces in
// any registered buffers (vortex's pool has one mmap per buffer,
// buf_pool.rs:92-98), 16-byte aligned, any lengths, the longest >= 2 chunks.
// Same rounds as batch_chunked, but each round's bytes are pulled by the
// gather kernel (vx_gather.hip) through the buffers' device mappings: lane m
// reads bytes [a, a + C) of its piece.
bool gather_batch(const vx_ctx* c, const uint8_t* const* ptrs, const uint32_t* lens, size_t n,
                  std::vector<const uint8_t*>& dev) {
    const uint64_t C = c->cfg.batch_chunk;
    if (n == 0 || C == 0 || c->slots[0].arena_cap < C) return false;
    uint32_t max_len = 0;
    dev.assign(n, nullptr);
    for (size_t i = 0; i < n; ++i) {
        if (lens[i] > c->cfg.max_piece_len) return false;
        max_len = std::max(max_len, lens[i]);
        if (lens[i] == 0) continue;
        if ((reinterpret_cast<uintptr_t>(ptrs[i]) & 15) || !is_registered(c, ptrs[i], lens[i], &dev[i]))
            return false;
    }
    return max_len >= 2 * C;
}

int batch_chunked_gather(vx_ctx* c, const uint32_t* lens, const uint8_t* expected, size_t n, uint8_t* matched_out,
                         uint8_t* digests_out, const std::vector<const uint8_t*>& dev) {
    const uint64_t C = c->cfg.batch_chunk;
    ChunkPipe cp(c);
    int rc = cp.open(n, expected, "batch");
    for (size_t i = 0; i < n; ++i) cp.bytes += lens[i];
    const Slot& s0 = c->slots[0];
    const uint64_t W = std::max<uint64_t>(1, std::min<uint64_t>(s0.cap, s0.arena_cap / C));
    // Pieces go longest first (stable, so equal lengths keep the caller's
    // order).  Every round is one C-byte chain whatever its lane count; in
    // caller-order windows every window with a long piece paid that whole
    // chain while its late rounds carried a few MiB each (config 3 from host,
    // DESIGN.md §6.4; that variant was removed in round 4, EXPERIMENTS.md).
    std::vector<uint32_t> order(n);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return lens[x] > lens[y]; });
    auto gather_copy = [&](uint32_t m, uint32_t tiles) {
        return [&, m, tiles](Slot& sl, hipStream_t st) -> int {
            if (hipMemcpyAsync(sl.d_src, sl.h_src, (size_t)m * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
                hipMemcpyAsync(sl.d_tfirst, sl.h_tfirst, (size_t)(m + 1) * 4, hipMemcpyHostToDevice, st) !=
                    hipSuccess)
                return fail(VX_EDEVICE, "batch: gather table H2D failed");
            hipError_t e = vx::launch_gather(sl.d_src, sl.d_offsets, sl.d_lens, sl.d_tfirst, m, tiles, sl.d_arena, st);
            if (e != hipSuccess) return hip_fail(e, "batch: gather launch");
            c->stats.gather_tiles += tiles;
            return 0;
        };
    };
    // Streaming rounds: a piece takes a lane from its first chunk to its
    // last, and new pieces (longest first) join any round until it holds
    // `target` bytes.  So the short pieces ride along the long pieces'
    // later rounds instead of queueing behind them, and no round is a
    // C-byte chain that moves only a few MiB.
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) total += lens[i];
    const uint64_t max_rounds = std::max<uint64_t>(1, (n ? (uint64_t)lens[order[0]] + C - 1 : 0) / C);
    // Spread evenly over the longest piece's rounds: a round is bound by
    // max(its bytes over PCIe, one C-byte chain), and the batch cannot take
    // fewer rounds than its longest piece has chunks.  (A uniform batch gets
    // target = n*C: every piece in the first round, as a window would.)
    const uint64_t target = std::max<uint64_t>(1, (total + max_rounds - 1) / max_rounds);
    std::vector<std::pair<uint32_t, uint64_t>> act, keep;  // (piece, next offset)
    size_t next = 0;
    while (!rc && (!act.empty() || next < n)) {
        const int si = cp.free_slot([] {});
        if (si < 0) {
            rc = si;
            break;
        }
        Slot& s = c->slots[si];
        reset_fill(s);
        uint32_t m = 0, tiles = 0;
        uint64_t bytes = 0;
        keep.clear();
        auto lane = [&](uint32_t i, uint64_t a) {
            const uint64_t L = lens[i];
            const uint32_t clen = (uint32_t)std::min<uint64_t>(C, L - a);
            s.h_offsets[m] = (uint64_t)m * C;
            s.h_lens[m] = clen;
            s.h_pidx[m] = i;
            s.h_poff[m] = a;
            s.h_tlen[m] = L;
            s.h_src[m] = clen ? reinterpret_cast<uint64_t>(dev[i] + a) : 0;
            tiles += clen ? vx::gather_tiles(clen) : 0;
            s.h_tfirst[m + 1] = tiles;
            ++m;
            bytes += clen;
            if (a + clen < L) keep.emplace_back(i, a + clen);
        };
        const bool continues = !act.empty();
        for (const auto& pa : act) lane(pa.first, pa.second);
        while (next < n && m < W && (bytes < target || m == 0)) lane(order[next++], 0);
        act.swap(keep);
        rc = cp.round(si, m, continues, true, gather_copy(m, tiles));
    }
    return cp.finish(matched_out, digests_out, rc);
}

// A host batch failed part way (an argument or allocation error at some
// submit, a failed launch, a device error).  The call borrows the caller's
// buffers only until it returns, so every slot still reading them — a DMA or
// the gather kernel in flight — is waited for, and every piece of the call
// is dropped: the filling slot is discarded without its deferred stage
// copies, completions already queued are cleared, and pending returns to 0
// (batch_impl starts with nothing pending), so later batches, vx_poll and
// vx_unregister_host_buffer see a clean context.
void abandon_batch(vx_ctx* c) {
    for (auto& s : c->slots)
        if (s.state == Slot::INFLIGHT) (void)hipEventSynchronize(s.done);
    for (auto& s : c->slots)
        if (s.state != Slot::FREE) {
            reset_fill(s);
            s.state = Slot::FREE;
        }
    c->done.clear();
    c->filling = -1;
    c->flush_pending = false;
    c->pending = 0;
}
}  // namespace

extern "C" {

static int batch_impl(vx_ctx* c, const uint8_t* const* ptrs, const uint32_t* lens, const uint8_t* expected, size_t n,
                      uint8_t* matched_out, uint8_t* digests_out) {
    if (!c) return fail(VX_EINVAL, "batch: NULL context");
    if (n && (!ptrs || !lens)) return fail(VX_EINVAL, "batch: NULL ptrs/lens");
    if (c->pending) return fail(VX_EBUSY, "batch: async pieces pending; drain and poll first");
    if (c->sticky) return c->sticky;
    if (c->filling >= 0) {  // an empty filling slot (pending == 0): hand it back
        c->slots[c->filling].state = Slot::FREE;
        c->filling = -1;
    }
    int rc = set_device(c);
    if (rc) return rc;
    uint64_t host_stride = 0;
    if (strided_batch(c, ptrs, lens, n, &host_stride))
        return batch_chunked(c, ptrs, lens, expected, n, matched_out, digests_out, host_stride);
    std::vector<const uint8_t*> dev;
    if (gather_batch(c, ptrs, lens, n, dev))
        return batch_chunked_gather(c, lens, expected, n, matched_out, digests_out, dev);
    std::vector<vx_completion> buf(1024);
    size_t got = 0;
    auto collect = [&]() -> int {
        for (;;) {
            int64_t k = vx_poll(c, buf.data(), buf.size());
            if (k < 0) return (int)k;
            for (int64_t j = 0; j < k; ++j) {
                const vx_completion& r = buf[j];
                if (digests_out) std::memcpy(digests_out + r.tag * 20, r.digest, 20);
                if (matched_out) matched_out[r.tag] = r.matched;
            }
            got += (size_t)k;
            if ((size_t)k < buf.size()) return 0;
        }
    };
    // Completions are harvested by acquire_filling when it runs out of slots;
    // polling here between submits would only add event queries to the
    // launch path, so the queue is drained only when it grows large.
    //
    // Pieces go in longest first and each slot fills to its capacity rather
    // than to batch_pieces (which vx_config_default sizes for max_piece_len
    // pieces).  A slot's kernel lasts as long as its longest piece's chain,
    // so in caller order a ragged batch put a long piece into almost every
    // small slot: config 3 from plain host memory ran at 2.1 GiB/s
    // (DESIGN.md §6.4).  Tags stay the caller's indices.
    for (size_t i = 0; i < n; ++i) {  // argument errors before anything is queued
        if (lens[i] > c->cfg.max_piece_len) return fail(VX_ERANGE, "batch: piece longer than max_piece_len");
        if (lens[i] && !ptrs[i]) return fail(VX_EINVAL, "batch: NULL piece pointer");
    }
    std::vector<uint32_t> order(n);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return lens[x] > lens[y]; });
    c->bulk = true;
    for (size_t p = 0; p < n; ++p) {
        const size_t i = order[p];
        rc = submit_impl(c, i, ptrs[i], lens[i], expected ? expected + i * 20 : nullptr);
        if (!rc && c->done.size() >= 65536) rc = collect();
        if (rc) break;
    }
    c->bulk = false;
    if (!rc) rc = vx_drain(c, 0);
    if (!rc) rc = collect();
    if (!rc && got != n) rc = fail(VX_EDEVICE, "batch: lost completions");
    if (rc) abandon_batch(c);
    return rc;
}

int vx_sha1_batch(vx_ctx* c, const uint8_t* const* ptrs, const uint32_t* lens, size_t n, uint8_t* digests_out) {
    if (!digests_out && n) return fail(VX_EINVAL, "vx_sha1_batch: NULL digests_out");
    return batch_impl(c, ptrs, lens, nullptr, n, nullptr, digests_out);
}

int vx_verify_batch(vx_ctx* c, const uint8_t* const* ptrs, const uint32_t* lens, const uint8_t* expected, size_t n,
                    uint8_t* matched_out, uint8_t* digests_out) {
    if (n && (!expected || !matched_out)) return fail(VX_EINVAL, "vx_verify_batch: NULL expected/matched_out");
    return batch_impl(c, ptrs, lens, expected, n, matched_out, digests_out);
}


// vx_verify_files_range, and with sp the engine's side of a split
// (vx_verify_files_split: pieces [sp->first, sp->end), always chunk rounds).
static int64_t verify_files_impl(vx_ctx* c, const char* const* paths, const uint64_t* file_lengths, size_t nfiles,
                                 uint32_t piece_length, const uint8_t* expected, size_t n_pieces, size_t first,
                                 size_t count, uint8_t* matched_out, uint32_t io_threads, vx_split* sp) {
    if (!c || (nfiles && (!paths || !file_lengths)) || piece_length == 0 || (n_pieces && !expected) ||
        (count && !matched_out))
        return fail(VX_EINVAL, "vx_verify_files: bad argument");
    if (first > n_pieces || count > n_pieces - first)
        return fail(VX_EINVAL, "vx_verify_files: piece range outside the torrent");
    if (c->sticky) return c->sticky;
    if (c->pending || c->filling >= 0) return fail(VX_EBUSY, "vx_verify_files: async pieces pending");
    uint64_t total = 0;
    for (size_t f = 0; f < nfiles; ++f) total += file_lengths[f];
    if (n_pieces != (total + piece_length - 1) / piece_length)
        return fail(VX_EINVAL, "vx_verify_files: n_pieces does not match the files' total length");
    if (count == 0) return 0;
    const uint64_t C = verify_chunk_for(c, count);
    bool chunked = piece_length >= 2 * C || sp;  // the split always streams chunk rounds
    if (piece_length > c->cfg.max_piece_len) chunked = true;  // whole pieces would not fit a slot
    if (chunked ? c->slots[0].arena_cap < std::min<uint64_t>(C, align_up(piece_length, vx_files::DirectIo::kBlock))
                : piece_length > c->cfg.max_piece_len)
        return fail(VX_ERANGE, "vx_verify_files: pieces do not fit the context's slots");
    int rc = set_device(c);
    if (rc) return rc;

    const uint64_t end = first + count;
    const uint64_t t_call = vx_files::Readers::now_ns();
    c->last_verify = vx_verify_trace{};
    c->last_rounds.clear();
    c->verify_t0_ns = t_call;
    const std::vector<vx_files::FileSpan> fs = vx_files::layout(file_lengths, nfiles, piece_length);
    std::vector<int> fds(nfiles, -1);
    for (size_t f = 0; f < nfiles; ++f) fds[f] = open(paths[f], O_RDONLY | O_CLOEXEC);
    const int nthreads = io_threads ? (int)io_threads : (int)std::max(1u, std::min(16u, usable_cpus()));
    std::vector<uint8_t> bad(count, 0);
    if (!sp) std::memset(matched_out, 0, count);  // (the split's pool writes its entries concurrently)
    {
        const vx_files::DirectIo dio(fds, c->cfg.direct_io != 0);
        vx_files::Readers rd(nthreads, fs, fds, piece_length, bad.data(), first, &dio);
        FileVerify fv{c, expected, matched_out, bad};
        c->harvest_counts_mismatches = false;
        // Uncached data: the disk binds, and takes bigger reads better.
        const uint64_t Cc = c->cfg.verify_cold_chunk;
        const uint64_t Cv = chunked && !c->cfg.verify_chunk && c->cfg.direct_io && Cc > C &&
                                    piece_length >= 2 * Cc && c->slots[0].arena_cap >= Cc &&
                                    dio.resident_fraction() < 0.5
                                ? Cc
                                : C;
        c->last_verify.chunk_bytes = chunked ? Cv : 0;
        uint64_t lowest = end;
        const int regime = c->cfg.direct_io && dio.resident_fraction() < 0.5 ? 1 : 0;  // the split's learned figures
        rc = sp        ? verify_split(fv, rd, sp, n_pieces, piece_length, total, Cv, &lowest, regime)
             : chunked ? verify_chunked(fv, rd, n_pieces, piece_length, total, first, end, Cv)
                       : verify_whole(fv, rd, n_pieces, piece_length, total, first, end);

        if (!rc && !chunked) {
            while (fv.done < count && !rc) {
                rc = reap(c, true);
                fv.consume();
                bool any = false;
                for (auto& s : c->slots) any |= s.state == Slot::INFLIGHT;
                if (!any && fv.done < count && !rc) rc = fail(VX_EDEVICE, "vx_verify_files: lost completions");
            }
        }
        c->harvest_counts_mismatches = true;
        vx_verify_trace& vt = c->last_verify;
        vt.read_busy_ms = rd.busy_ns() * 1e-6;
        vt.read_bytes = rd.bytes_read();
        vt.direct_bytes = dio.direct_bytes();
        vt.readers = (uint32_t)rd.threads();
        if (rd.first_start_ns()) {
            vt.read_span_ms = (rd.last_end_ns() - rd.first_start_ns()) * 1e-6;
            vt.first_read_ms = (rd.first_end_ns() - t_call) * 1e-6;
        }
        if (rc) {
            // The call fails and its results are dropped: wait for every slot
            // still reading the stages, then free them without harvest(), so
            // abandoned pieces never reach vx_stats.
            for (auto& s : c->slots)
                if (s.state == Slot::INFLIGHT) (void)hipEventSynchronize(s.done);
            for (auto& s : c->slots)
                if (s.state == Slot::INFLIGHT) {
                    reset_fill(s);
                    s.state = Slot::FREE;
                }
            c->done.clear();
        }
    }
    for (int fd : fds)
        if (fd >= 0) close(fd);
    c->last_verify.wall_ms = (vx_files::Readers::now_ns() - t_call) * 1e-6;
    if (rc) return rc;
    int64_t nbad = 0;
    for (uint8_t x : bad) nbad += x;
    c->stats.io_errors += (uint64_t)nbad;
    return nbad;
}

int64_t vx_verify_files_range(vx_ctx* c, const char* const* paths, const uint64_t* file_lengths, size_t nfiles,
                              uint32_t piece_length, const uint8_t* expected, size_t n_pieces, size_t first,
                              size_t count, uint8_t* matched_out, uint32_t io_threads) {
    return verify_files_impl(c, paths, file_lengths, nfiles, piece_length, expected, n_pieces, first, count,
                             matched_out, io_threads, nullptr);
}

int vx_split_init(vx_split* s, uint64_t first, uint64_t end, uint32_t cpu_threads, double cpu_thread_rate) {
    if (!s || first > end || end > 0xffffffffull) return fail(VX_EINVAL, "vx_split_init: bad range");
    if (!(cpu_thread_rate >= 0)) return fail(VX_EINVAL, "vx_split_init: cpu_thread_rate must be >= 0");
    *s = vx_split{};
    s->first = first;
    s->end = end;
    s->cpu_threads = cpu_threads;
    s->cpu_thread_rate = cpu_thread_rate;
    s->start_ns = vx_files::Readers::now_ns();
    __atomic_store_n(&s->word, first | (end << 32), __ATOMIC_RELEASE);
    return 0;
}

int64_t vx_split_claim(vx_split* s) {
    if (!s) return -1;
    uint64_t w = __atomic_load_n(&s->word, __ATOMIC_ACQUIRE);
    for (;;) {
        const uint64_t head = w & 0xffffffffull, stop = w >> 32;
        if (head >= stop) return -1;
        if (__atomic_compare_exchange_n(&s->word, &w, w + 1, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE))
            return (int64_t)head;
    }
}

void vx_split_done(vx_split* s, uint64_t pieces) {
    if (!s) return;
    // the latest verdict's time (a later one never moves it back), published
    // with the count
    const uint64_t t = vx_files::Readers::now_ns();
    uint64_t was = __atomic_load_n(&s->pool_last_ns, __ATOMIC_RELAXED);
    while (was < t &&
           !__atomic_compare_exchange_n(&s->pool_last_ns, &was, t, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
    }
    __atomic_fetch_add(&s->pool_done, pieces, __ATOMIC_RELEASE);
}

uint64_t vx_split_boundary(const vx_split* s) {
    return s ? __atomic_load_n(&s->word, __ATOMIC_ACQUIRE) >> 32 : 0;
}

int64_t vx_verify_files_split(vx_ctx* c, const char* const* paths, const uint64_t* file_lengths, size_t nfiles,
                              uint32_t piece_length, const uint8_t* expected, size_t n_pieces, vx_split* s,
                              uint8_t* matched_out, uint32_t io_threads) {
    if (!s || s->first > s->end || s->end > n_pieces) return fail(VX_EINVAL, "vx_verify_files_split: bad split");
    return verify_files_impl(c, paths, file_lengths, nfiles, piece_length, expected, n_pieces, s->first,
                             s->end - s->first, matched_out, io_threads, s);
}

int64_t vx_verify_files(vx_ctx* c, const char* const* paths, const uint64_t* file_lengths, size_t nfiles,
                        uint32_t piece_length, const uint8_t* expected, size_t n_pieces, uint8_t* matched_out,
                        uint32_t io_threads) {
    return vx_verify_files_range(c, paths, file_lengths, nfiles, piece_length, expected, n_pieces, 0, n_pieces,
                                 matched_out, io_threads);
}

// In-process multi-device re-verify: vortex is ONE process
// with one event loop (event_loop.rs:385), so where torch.distributed would
// run one process per GPU, a Rust caller holds one context per GPU and this
// call splits [0, n_pieces) across them by the same contiguous rule as
// vortex_amd.shard.shard_range (n/nctx each, remainder to the last
// contexts), one host thread per context.  Each thread runs
// vx_verify_files_range on its context and writes its slice of matched_out
// in place, so no merge step is needed.
int64_t vx_verify_files_multi(vx_ctx* const* ctxs, size_t nctx, const char* const* paths,
                              const uint64_t* file_lengths, size_t nfiles, uint32_t piece_length,
                              const uint8_t* expected, size_t n_pieces, uint8_t* matched_out, uint32_t io_threads) {
    if (!ctxs || nctx == 0 || nctx > 1024) return fail(VX_EINVAL, "vx_verify_files_multi: bad context list");
    for (size_t k = 0; k < nctx; ++k) {
        if (!ctxs[k]) return fail(VX_EINVAL, "vx_verify_files_multi: NULL context");
        for (size_t j = 0; j < k; ++j)
            if (ctxs[j] == ctxs[k]) return fail(VX_EINVAL, "vx_verify_files_multi: a context appears twice");
    }
    if (n_pieces && (!expected || !matched_out)) return fail(VX_EINVAL, "vx_verify_files_multi: bad argument");
    const uint32_t total_io = io_threads ? io_threads : std::max(1u, std::min(16u, usable_cpus()));
    const uint32_t per_ctx = std::max<uint32_t>(1, total_io / (uint32_t)nctx);
    const size_t base = n_pieces / nctx, rem = n_pieces % nctx, extra_from = nctx - rem;
    std::vector<int64_t> rcs(nctx, 0);
    std::vector<std::string> errs(nctx);
    auto run = [&](size_t k) {
        const size_t first = k * base + (k > extra_from ? k - extra_from : 0);
        const size_t count = base + (k >= extra_from ? 1 : 0);
        rcs[k] = vx_verify_files_range(ctxs[k], paths, file_lengths, nfiles, piece_length, expected, n_pieces,
                                       first, count, matched_out + first, per_ctx);
        if (rcs[k] < 0) errs[k] = g_err;  // g_err is thread-local
    };
    std::vector<std::thread> th;
    th.reserve(nctx);
    size_t started = 1;
    try {
        for (; started < nctx; ++started) th.emplace_back(run, started);
    } catch (...) {  // could not start a thread: run the rest on this one
    }
    run(0);
    for (size_t k = started; k < nctx; ++k) run(k);
    for (auto& t : th) t.join();
    int64_t nbad = 0;
    for (size_t k = 0; k < nctx; ++k) {
        if (rcs[k] < 0) {
            g_err = "context " + std::to_string(k) + ": " + errs[k];
            return rcs[k];
        }
        nbad += rcs[k];
    }
    return nbad;
}

// The split over several GPUs of one process: one host thread per context,
// each running vx_verify_files_split on the same claim word, which is
// declared for nctx engines so each sizes its groups as one of nctx equal
// takers beside the pool.  io_threads is the total reader count, divided.
int64_t vx_verify_files_split_multi(vx_ctx* const* ctxs, size_t nctx, const char* const* paths,
                                    const uint64_t* file_lengths, size_t nfiles, uint32_t piece_length,
                                    const uint8_t* expected, size_t n_pieces, vx_split* s, uint8_t* matched_out,
                                    uint32_t io_threads) {
    if (!ctxs || nctx == 0 || nctx > 1024 || !s) return fail(VX_EINVAL, "vx_verify_files_split_multi: bad argument");
    for (size_t k = 0; k < nctx; ++k) {
        if (!ctxs[k]) return fail(VX_EINVAL, "vx_verify_files_split_multi: NULL context");
        for (size_t j = 0; j < k; ++j)
            if (ctxs[j] == ctxs[k]) return fail(VX_EINVAL, "vx_verify_files_split_multi: a context appears twice");
    }
    s->engines = (uint32_t)nctx;
    const uint32_t total_io = io_threads ? io_threads : std::max(1u, std::min(16u, usable_cpus()));
    const uint32_t per_ctx = std::max<uint32_t>(1, total_io / (uint32_t)nctx);
    std::vector<int64_t> rcs(nctx, 0);
    std::vector<std::string> errs(nctx);
    auto run = [&](size_t k) {
        rcs[k] = vx_verify_files_split(ctxs[k], paths, file_lengths, nfiles, piece_length, expected, n_pieces, s,
                                       matched_out, per_ctx);
        if (rcs[k] < 0) errs[k] = g_err;  // g_err is thread-local
    };
    std::vector<std::thread> th;
    th.reserve(nctx);
    size_t started = 1;
    try {
        for (; started < nctx; ++started) th.emplace_back(run, started);
    } catch (...) {  // could not start a thread: run the rest on this one
    }
    run(0);
    for (size_t k = started; k < nctx; ++k) run(k);
    for (auto& t : th) t.join();
    int64_t nbad = 0;
    for (size_t k = 0; k < nctx; ++k) {
        if (rcs[k] < 0) {
            g_err = "context " + std::to_string(k) + ": " + errs[k];
            return rcs[k];
        }
        nbad += rcs[k];
    }
    return nbad;
}

int vx_sha1_device_uniform_variant(const void* d_base, uint64_t stride, uint32_t len, uint32_t n, void* d_digests,
                                   const void* d_expected, void* d_matched, void* stream, int variant) {
    if (n == 0) return 0;
    if (!d_base) return fail(VX_EINVAL, "vx_sha1_device_uniform: NULL base");
    if (!d_digests && !(d_expected && d_matched))
        return fail(VX_EINVAL, "vx_sha1_device_uniform: need d_digests or d_expected+d_matched");
    if (d_matched && !d_expected) return fail(VX_EINVAL, "vx_sha1_device_uniform: d_matched needs d_expected");
    if ((reinterpret_cast<uintptr_t>(d_base) & 15) || (stride & 15))
        return fail(VX_EINVAL, "vx_sha1_device_uniform: base and stride must be 16-byte aligned");
    if (n > 1 && stride < len) return fail(VX_EINVAL, "vx_sha1_device_uniform: stride < len");
    if (variant < 0 || variant > 4)
        return fail(VX_EINVAL, "vx_sha1_device_uniform: unknown variant");
    hipError_t e = vx::launch_uniform(static_cast<const uint8_t*>(d_base), stride, len, n,
                                      static_cast<uint8_t*>(d_digests), static_cast<const uint8_t*>(d_expected),
                                      static_cast<uint8_t*>(d_matched), static_cast<hipStream_t>(stream), variant);
    if (e != hipSuccess) return hip_fail(e, "sha1 uniform kernel launch");
    return 0;
}

int vx_sha1_device_uniform(const void* d_base, uint64_t stride, uint32_t len, uint32_t n, void* d_digests,
                           const void* d_expected, void* d_matched, void* stream) {
    return vx_sha1_device_uniform_variant(d_base, stride, len, n, d_digests, d_expected, d_matched, stream, 0);
}

int vx_sha1_device_ragged_variant(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lens,
                                  const uint32_t* d_order, uint32_t n, void* d_digests, const void* d_expected,
                                  void* d_matched, void* stream, int variant) {
    if (n == 0) return 0;
    if (!d_base || !d_offsets || !d_lens) return fail(VX_EINVAL, "vx_sha1_device_ragged: NULL argument");
    if (!d_digests && !(d_expected && d_matched))
        return fail(VX_EINVAL, "vx_sha1_device_ragged: need d_digests or d_expected+d_matched");
    if (d_matched && !d_expected) return fail(VX_EINVAL, "vx_sha1_device_ragged: d_matched needs d_expected");
    if (reinterpret_cast<uintptr_t>(d_base) & 15)
        return fail(VX_EINVAL, "vx_sha1_device_ragged: base must be 16-byte aligned");
    if (variant < 0 || variant > vx::kSplitWide) return fail(VX_EINVAL, "vx_sha1_device_ragged: unknown variant");
    hipError_t e = vx::launch_ragged(static_cast<const uint8_t*>(d_base), d_offsets, d_lens, d_order, n,
                                     static_cast<uint8_t*>(d_digests), static_cast<const uint8_t*>(d_expected),
                                     static_cast<uint8_t*>(d_matched), static_cast<hipStream_t>(stream), variant);
    if (e != hipSuccess) return hip_fail(e, "sha1 ragged kernel launch");
    return 0;
}

int vx_sha1_device_ragged(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lens,
                          const uint32_t* d_order, uint32_t n, void* d_digests, const void* d_expected,
                          void* d_matched, void* stream) {
    return vx_sha1_device_ragged_variant(d_base, d_offsets, d_lens, d_order, n, d_digests, d_expected, d_matched,
                                         stream, 0);
}

int vx_sha1_device_ragged_hint(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lens,
                               const uint32_t* d_order, uint32_t n, uint32_t max_len, uint64_t total_len,
                               void* d_digests, const void* d_expected, void* d_matched, void* stream) {
    return vx_sha1_device_ragged_variant(d_base, d_offsets, d_lens, d_order, n, d_digests, d_expected, d_matched,
                                         stream, vx::plan_ragged(n, max_len, total_len));
}

// Host-only cost model of a bulk verify.  One piece is one
// lane and SHA-1 is Merkle-Damgård, so a piece of L bytes is a chain of
// blocks(L) dependent compressions at kChainBlock seconds each on the split
// kernels (the chunked re-verify pipelines its rounds, so the chain, not the
// round count, is what remains); the bytes cross PCIe at kPcieRate.  The call
// takes the larger of the two, a fixed setup, and a fraction of the smaller
// (they overlap, but not perfectly).  The caller's pool: ceil(n / threads)
// rounds of one piece per thread at cpu_thread_rate bytes/s (rayon runs one
// piece per task, torrent.rs:724-740).  Fitted to the grid measured by
// tools/crossover_grid.py on the asm-consumer build
// (profiles/r02/crossover/grid.json: 22 points, 2-16 MiB x 64-4,096 pieces;
// GPU predictions within 5 %); tests/test_abi.py checks the fit and every
// decision against that file.  use_gpu asks for a 10 % margin: near a tie the
// caller's own pool is the safe choice.
int vx_plan_verify(uint64_t n_pieces, uint32_t piece_length, uint64_t total_length, uint32_t cpu_threads,
                   double cpu_thread_rate, vx_plan* out) {
    return vx_plan_verify_gpus(n_pieces, piece_length, total_length, cpu_threads, cpu_thread_rate, 1, out);
}

// The same model over n_gpus contexts (vx_verify_files_multi):
// each GPU's share of the bytes crosses its own PCIe link, so the transfer
// term divides by n_gpus; one piece's chain does not shrink, which is why a
// host with many cores can keep its pool against any number of GPUs when the
// pieces are long (INTEGRATION.md "A whole node is a different host").
namespace {
constexpr double kSetup = 1.5e-3;
constexpr double kOverlapLoss = 0.08, kMargin = 1.1;
constexpr double kBatchLatency = 1e-3;  // launch, H2D of a small batch, D2H, poll
// A split runs the GPU side's reads beside the pool's hashing on the same
// host.  The pool is sized to leave the engine's readers their cores (the
// caller passes its size; 12 of 16 threads beside 8 readers measured stable);
// beside the engine it hashes at kSplitPool of its per-thread rate alone, and
// the GPU side's bytes move at kSplitLink of the link rate (page-cache reads,
// stage writes and the DMA share host memory with the pool's hashing).  Fitted
// to the warm config-5 split over three boxes (profiles/r05/split/: GPU side
// 36-43 GB/s, the 12-thread pool at 0.85-0.98 of its rate alone), then refit
// on four HEAD bench runs with the copy stream and huge-page stages
// (refit_r05_bench.json: GPU side 38-39.5 GiB/s at its largest share, the pool
// at 0.74-0.85 of its rate alone, median 0.80; at 0.85 the point with 10 % more
// GPU pieces won on all four, by 1-16 %).
constexpr double kSplitLink = 0.74, kSplitPool = 0.80;

// The GPU path over `bytes` bytes of pieces piece_length long, over n_gpus links
// at `link` of the PCIe rate.
void plan_gpu(double L, double bytes, uint32_t n_gpus, vx_plan* out, double link = 1.0) {
    out->gpu_chain_s = std::ceil((L + 9) / 64) * kChainBlock;
    out->gpu_transfer_s = bytes / (kPcieRate * link) / std::max<uint32_t>(1, n_gpus);
    out->gpu_s = std::max(out->gpu_transfer_s, out->gpu_chain_s) + kSetup +
                 kOverlapLoss * std::min(out->gpu_transfer_s, out->gpu_chain_s);
}
}  // namespace

int vx_plan_verify_gpus(uint64_t n_pieces, uint32_t piece_length, uint64_t total_length, uint32_t cpu_threads,
                        double cpu_thread_rate, uint32_t n_gpus, vx_plan* out) {
    if (!out || piece_length == 0) return fail(VX_EINVAL, "vx_plan_verify: bad argument");
    if (n_pieces != (total_length + piece_length - 1) / piece_length)
        return fail(VX_EINVAL, "vx_plan_verify: n_pieces does not match total_length");
    const double threads = cpu_threads ? cpu_threads : 16;
    const double rate = cpu_thread_rate > 0 ? cpu_thread_rate : 2.2e9;
    const double L = piece_length;
    *out = vx_plan{};
    if (n_pieces == 0) return 0;
    plan_gpu(L, (double)total_length, n_gpus, out);
    out->cpu_s = std::ceil((double)n_pieces / threads) * (L / rate);
    out->piece_latency_s = out->gpu_chain_s + kBatchLatency;
    out->cpu_piece_latency_s = L / rate;
    out->use_gpu = out->gpu_s * kMargin < out->cpu_s ? 1 : 0;
    return 0;
}

// The split of one bulk verify between the GPUs (the tail of the piece range)
// and the caller's pool (the head), run at once: the GPU side's time is the
// model above over its bytes at kSplitLink of the link; the pool's is its
// pieces in rounds of one piece per thread.  Every split k = 0..n is scored by
// the slower side and the fastest wins; unless it beats the pool alone by
// kMargin the pool keeps everything.
int vx_plan_verify_split(uint64_t n_pieces, uint32_t piece_length, uint64_t total_length, uint32_t cpu_threads,
                         double cpu_thread_rate, uint32_t n_gpus, uint64_t* gpu_first, uint64_t* gpu_count,
                         vx_plan* out) {
    if (!gpu_first || !gpu_count || piece_length == 0) return fail(VX_EINVAL, "vx_plan_verify_split: bad argument");
    if (n_pieces != (total_length + piece_length - 1) / piece_length)
        return fail(VX_EINVAL, "vx_plan_verify_split: n_pieces does not match total_length");
    const double threads = cpu_threads ? cpu_threads : 16;
    const double rate = cpu_thread_rate > 0 ? cpu_thread_rate : 2.2e9;
    const double L = piece_length;
    const double last = n_pieces ? (double)(total_length - (n_pieces - 1) * (uint64_t)piece_length) : 0.0;
    auto gpu_bytes = [&](uint64_t k) { return k ? (double)(k - 1) * L + last : 0.0; };
    auto cpu_time = [&](uint64_t k) {  // the pool's n - k pieces, one per thread per round
        if (k >= n_pieces) return 0.0;
        return std::ceil((double)(n_pieces - k) / threads) * (L / (k ? rate * kSplitPool : rate));
    };
    vx_plan g{};
    auto gpu_time = [&](uint64_t k) {
        plan_gpu(L, gpu_bytes(k), n_gpus, &g, k < n_pieces ? kSplitLink : 1.0);
        return g.gpu_s;
    };
    uint64_t best_k = 0;
    double best_t = cpu_time(0);
    const double pool_alone = best_t;
    auto consider = [&](uint64_t k) {
        if (k < 1 || k > n_pieces) return;
        const double t = std::max(gpu_time(k), cpu_time(k));
        if (t < best_t || (t == best_t && k < best_k)) best_t = t, best_k = k;
    };
    // On 1 <= k < n the GPU side's time never falls as k grows and the
    // pool's never rises, so the slower side is least where they cross:
    // bisect for the first k whose GPU time reaches the pool's, then score it,
    // its neighbours and k = n (whose link has no pool beside it).  A scan of
    // every k cost a multi-TB torrent of 16 KiB pieces ~10^7 evaluations.
    if (n_pieces > 1) {
        uint64_t lo = 1, hi = n_pieces - 1;
        if (gpu_time(hi) < cpu_time(hi)) {
            lo = hi;
        } else {
            while (lo < hi) {
                const uint64_t mid = lo + (hi - lo) / 2;
                if (gpu_time(mid) >= cpu_time(mid)) hi = mid;
                else lo = mid + 1;
            }
        }
        for (uint64_t k = lo > 2 ? lo - 2 : 1; k <= std::min<uint64_t>(n_pieces - 1, lo + 2); ++k) consider(k);
        // left of the crossing the pool's side binds, and its time is a step
        // function (rounds of `threads` pieces): the step's first k ties it
        if (lo > 1) {
            const uint64_t m = (uint64_t)std::ceil((double)(n_pieces - (lo - 1)) / threads);
            const uint64_t k0 = n_pieces > m * (uint64_t)threads ? n_pieces - m * (uint64_t)threads : 1;
            consider(std::max<uint64_t>(1, k0));
        }
    }
    consider(n_pieces);
    if (best_k && best_t * kMargin >= pool_alone) best_k = 0;
    *gpu_count = best_k;
    *gpu_first = n_pieces - best_k;
    if (out) {
        *out = vx_plan{};
        if (best_k) plan_gpu(L, gpu_bytes(best_k), n_gpus, out, best_k < n_pieces ? kSplitLink : 1.0);
        out->cpu_s = cpu_time(best_k);
        vx_plan one{};
        plan_gpu(L, L, 1, &one);  // the download path's figures do not depend on the split
        out->piece_latency_s = one.gpu_chain_s + kBatchLatency;
        out->cpu_piece_latency_s = L / rate;
        out->use_gpu = best_k ? 1 : 0;
    }
    return 0;
}

int vx_get_stats(const vx_ctx* c, vx_stats* out) {
    if (!c || !out) return fail(VX_EINVAL, "vx_get_stats: NULL argument");
    *out = c->stats;
    return 0;
}

int vx_reset_stats(vx_ctx* c) {
    if (!c) return fail(VX_EINVAL, "vx_reset_stats: NULL context");
    c->stats = vx_stats{};
    return 0;
}

int vx_last_verify(const vx_ctx* c, vx_verify_trace* out) {
    if (!c || !out) return fail(VX_EINVAL, "vx_last_verify: NULL argument");
    *out = c->last_verify;
    return 0;
}

int64_t vx_last_verify_rounds(const vx_ctx* c, vx_verify_round* out, size_t max) {
    if (!c || (max && !out)) return fail(VX_EINVAL, "vx_last_verify_rounds: NULL argument");
    const size_t k = std::min(max, c->last_rounds.size());
    if (k) std::memcpy(out, c->last_rounds.data(), k * sizeof(vx_verify_round));
    return (int64_t)c->last_rounds.size();
}

int vx_tuning_zero_copy_plan(uint32_t n, uint64_t total_len) {
    (void)total_len;  // the policy no longer depends on the slot's bytes (kept in the signature)
    return zc_loader_wins(n) ? 2 : 1;
}

int vx_tuning_zero_copy_kernel(const uint64_t* d_srcs, const uint32_t* d_lens, uint32_t n, void* d_digests,
                               const void* d_expected, void* d_matched, int loader, void* stream) {
    if (n && (!d_srcs || !d_lens || !d_digests)) return fail(VX_EINVAL, "vx_tuning_zero_copy_kernel: NULL argument");
    if ((d_expected == nullptr) != (d_matched == nullptr))
        return fail(VX_EINVAL, "vx_tuning_zero_copy_kernel: expected and matched go together");
    hipError_t e = vx::launch_zero_copy(d_srcs, d_lens, n, static_cast<uint8_t*>(d_digests),
                                        static_cast<const uint8_t*>(d_expected), static_cast<uint8_t*>(d_matched),
                                        loader != 0, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : hip_fail(e, "vx_tuning_zero_copy_kernel");
}
#ifdef VX_TEST_HOOKS
void vx_tuning_fail_submit_after(vx_ctx* c, int64_t k) {
    if (c) c->fail_submit_after = k < 0 ? -1 : k;
}
void vx_tuning_fail_launch_after(vx_ctx* c, int64_t k) {
    if (c) c->fail_launch_after = k < 0 ? -1 : k;
}
void vx_tuning_verify_copy_stream(vx_ctx* c, int mode) {
    if (c) c->verify_copy_stream = mode ? 1 : 0;
}
void vx_tuning_split_rules(vx_ctx* c, int one_round, uint64_t round_cap, int lag, int learn) {
    if (!c) return;
    c->split_lag_on = lag ? 1 : 0;
    c->split_learn = learn ? 1 : 0;
    c->split_one_round = one_round == 2 ? 2 : one_round ? 1 : 0;
    c->split_round_cap = round_cap;
}
void vx_tuning_stage_huge(vx_ctx* c, int on) {
    if (!c) return;
    c->stage_huge = on ? 1 : 0;
    if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);  // no copy still reads a stage
    for (auto& s : c->slots)  // reallocated on next use (every slot is idle between calls)
        if (s.state == Slot::FREE) free_stage(s);
}
#endif
uint64_t vx_tuning_split_take_tail(vx_split* s, uint64_t k, uint64_t* was) {
    return s ? split_take_tail(s, k, UINT64_MAX, was) : 0;
}
size_t vx_tuning_last_split(const vx_ctx* c, double* out, size_t max) {
    if (!c) return 0;
    const size_t k = std::min(max, c->last_split.size());
    for (size_t i = 0; i < k && out; ++i) {
        const auto& d = c->last_split[i];
        const double row[13] = {d.t_ms, d.pool_rate, d.engine_rate, d.block_ns, d.t_engine_ms, d.t_pool_ms,
                                (double)d.unclaimed, (double)d.group, (double)d.lanes, (double)d.pool_done,
                                (double)d.mode, (double)d.measured, d.lag_ms};
        std::memcpy(out + 13 * i, row, sizeof row);
    }
    return c->last_split.size();
}
size_t vx_tuning_chunk_schedule(uint64_t L, uint64_t C, int head, int tail, uint64_t* out, size_t max) {
    if (C < 4 || C % 4) return 0;
    const auto r = chunk_schedule(L, C, std::max(0, std::min(5, head)), std::max(0, std::min(5, tail)));
    for (size_t i = 0; i < r.size() && i < max && out; ++i) {
        out[2 * i] = r[i].first;
        out[2 * i + 1] = r[i].second;
    }
    return r.size();
}

int vx_tuning_plan_ragged(uint32_t n, uint32_t max_len, uint64_t total_len) {
    return vx::plan_ragged(n, max_len, total_len);
}

int vx_sort_order(const uint32_t* lens, uint32_t n, uint32_t* order_out) {
    if (n && (!lens || !order_out)) return fail(VX_EINVAL, "vx_sort_order: NULL argument");
    std::iota(order_out, order_out + n, 0u);
    std::stable_sort(order_out, order_out + n, [lens](uint32_t a, uint32_t b) { return lens[a] > lens[b]; });
    return 0;
}

int vx_synth_fill(void* d_base, uint64_t stride, uint32_t len, uint32_t n, uint64_t first, uint64_t seed,
                  uint32_t corrupt_every, void* stream) {
    if (n == 0) return 0;
    if (!d_base) return fail(VX_EINVAL, "vx_synth_fill: NULL base");
    if ((reinterpret_cast<uintptr_t>(d_base) & 15) || (stride & 15) || (n > 1 && stride < len))
        return fail(VX_EINVAL, "vx_synth_fill: base/stride must be 16-byte aligned and stride >= len");
    hipError_t e = vx::launch_synth_fill(static_cast<uint8_t*>(d_base), stride, len, n, first, seed, corrupt_every,
                                         static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "synth launch");
    return 0;
}

}  // extern "C"
