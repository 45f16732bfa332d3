/*
 * vx_hash.h — C ABI of the MI355X SHA-1 piece-verification engine.
 *
 * This is the drop-in boundary for vortex's "Parallel hash computations" pool.
 * In the reference the boundary is not a trait but an inline closure handed to
 * rayon plus an mpsc channel back to the event loop:
 *
 *   submit   bittorrent/src/peer_comm/peer_connection.rs:1145-1158
 *            scope.spawn(move |_| { Sha1 over buffer[..piece_len];
 *                                   == metadata.pieces[index];
 *                                   complete_tx.send(DownloadedPiece{..}) })
 *   complete bittorrent/src/torrent.rs:415-442
 *            while let Ok(p) = downloaded_piece_rc.try_recv() { .. }
 *   bulk     bittorrent/src/torrent.rs:724-740 (par_iter over all pieces,
 *            each bittorrent/src/file_store.rs:228-303 check_piece_hash_sync)
 *   record   bittorrent/src/piece_selector.rs:311-317 (DownloadedPiece)
 *
 * Every entry point below names the reference interface it replaces.  The
 * signatures use only plain pointers, sizes and integers so that Rust
 * (`extern "C"`), ctypes, cgo or JNI can bind them directly; INTEGRATION.md
 * shows the Rust binding.
 *
 * Conventions
 *  - Return codes are 0 on success or a negative errno-style VX_E* value.  A
 *    hash mismatch is NOT an error: it is reported as matched = 0, exactly as
 *    the reference reports hash_matched = false.  No function aborts or throws
 *    across the ABI; vx_last_error() gives a thread-local message.
 *  - Digests are the 20-byte big-endian SHA-1 output (what
 *    `Sha1::finalize().as_slice()` returns), stored back to back.
 *  - Threading (mirrors the reference): one thread (the io_uring event-loop
 *    thread) submits and the same thread polls.  A vx_ctx is not internally
 *    synchronised; internal HIP streams are invisible to the caller.
 *    Separate contexts (e.g. one per torrent) share nothing but the device
 *    and may be driven from different threads concurrently
 *    (tests/test_gpu_parity.py::test_two_contexts_two_threads).
 *  - Device entry points (vx_sha1_device_*) take device pointers and a HIP
 *    stream (hipStream_t passed as void*; NULL = the null stream) and only
 *    enqueue work: they return before the kernel finishes.
 */
#ifndef VX_HASH_H
#define VX_HASH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VX_ABI_VERSION 3

/* Error codes (negative errno values). */
#define VX_OK 0
#define VX_EINVAL (-22)  /* bad argument (null pointer, n/len out of range, misalignment) */
#define VX_ENOMEM (-12)  /* host or device allocation failed */
#define VX_ERANGE (-34)  /* piece longer than the context's max_piece_len */
#define VX_ENODEV (-19)  /* no such HIP device */
#define VX_EDEVICE (-5)  /* a HIP runtime call failed (see vx_last_error) */
#define VX_EBUSY (-16)   /* operation not allowed while work is in flight */

#define VX_DIGEST_LEN 20

/* Device batch layout: piece bytes live in one device allocation; piece i
 * starts at base + offsets[i] (uniform batches: base + i*stride).  Piece
 * starts must be 16-byte aligned (the kernels load 16 bytes per lane);
 * lengths are arbitrary (0 .. 4 GiB-1). */

/* One completion, the C form of DownloadedPiece (piece_selector.rs:311-317):
 * `tag` is whatever the caller passed to vx_submit (vortex packs the piece
 * index and the ConnectionId into it), `matched` is hash_matched.  The Buffer
 * member has no C counterpart: the caller keeps the buffer and gets it back
 * by tag. */
typedef struct vx_completion {
    uint64_t tag;
    uint8_t matched;
    uint8_t digest[VX_DIGEST_LEN];
    uint8_t _pad[3];
} vx_completion;

/* Everything a caller may choose is here; the engine reads no environment
 * variables.  Start from vx_config_default() and change fields (ABI 2 added
 * the six after slot_bytes; vx_create rejects values outside their ranges,
 * chunk sizes above 1 GiB included). */
typedef struct vx_config {
    int32_t device;             /* HIP device ordinal                                   */
    uint32_t max_piece_len;     /* bytes; torrent piece_length (torrent.rs:344 pool size) */
    uint32_t batch_pieces;      /* launch a batch once this many pieces are queued      */
    uint32_t slots;             /* batches in flight (each has its own stream + arena)  */
    uint64_t slot_bytes;        /* device arena bytes per slot (>= max_piece_len)       */
    uint32_t zero_copy;         /* 1 (default): a batch whose pieces are all registered and 16-byte aligned is
                                 * hashed straight out of host memory; 0: such pieces are gathered into HBM first */
    uint32_t direct_io;         /* re-verify: 1 (default) reads uncached, 4 KiB-aligned ranges with O_DIRECT;
                                 * 0: every read through the page cache (vortex's own pread)                   */
    uint32_t batch_chunk;       /* host batches of long pieces: bytes per resumable round (default 65536,
                                 * multiple of 4096); 0: whole pieces per slot                                  */
    uint32_t verify_chunk;      /* re-verify: bytes per resumable round (multiple of 4096); 0 (default): chosen
                                 * per call, 256 KiB when one window holds every piece, else 128 KiB           */
    uint32_t verify_cold_chunk; /* re-verify of data not in the page cache: bytes per round (multiple of 4096);
                                 * 0 (default): as when cached                                                  */
    uint32_t verify_ramp;       /* re-verify: first and last rounds shrink to chunk / 2^(d+1), d = 0..5
                                 * (default 1; 0: no ramp)                                                      */
    uint32_t refuse_when_full;  /* (ABI 3) async submits: 0 (default) wait for the oldest batch when every slot
                                 * is in flight; 1: return VX_EBUSY instead, the piece NOT taken, so the event
                                 * loop never blocks and hands the piece to its own pool (the overflow)      */
} vx_config;

typedef struct vx_ctx vx_ctx;

/* ---- library ---------------------------------------------------------- */
int vx_abi_version(void);
const char* vx_last_error(void);
const char* vx_strerror(int code);
/* Number of HIP devices (0 when no GPU or no driver). */
int vx_device_count(void);
/* Fill *cfg with defaults for a torrent whose piece_length is max_piece_len. */
void vx_config_default(vx_config* cfg, uint32_t max_piece_len);

/* ---- context: replaces InitializedState's downloaded_piece_tx/rc pair and
 *      the rayon scope it feeds (torrent.rs:319-320, 333; event_loop.rs:385) */
int vx_create(const vx_config* cfg, vx_ctx** out);
/* Drains all in-flight work first (the reference's scope joins every spawned
 * hash before EventLoop::run returns, event_loop.rs:385-602), then frees.
 * On a failed context it waits for the device to stop (every stream) before
 * unregistering host buffers, so borrowed buffers are free once it returns. */
int vx_destroy(vx_ctx* ctx);

/* Pin and device-map a host range (e.g. a BufferPool's AnonymousMmap,
 * buf_ring.rs:24-42) so pieces inside it reach the GPU without an internal
 * pinned copy: any batch slot whose pieces are all registered and 16-byte
 * aligned — async, or a host batch of short pieces — is hashed by a kernel
 * that reads them over PCIe itself (zero-copy slots, vx_config.zero_copy);
 * host batches of long pieces pull them with one gather kernel per resumable
 * round.  Ranges must not overlap. */
int vx_register_host_buffer(vx_ctx* ctx, void* ptr, size_t len);
int vx_unregister_host_buffer(vx_ctx* ctx, void* ptr);

/* ---- async download path ---------------------------------------------- */
/* Replaces `scope.spawn(hash closure)` (peer_connection.rs:1145-1158).
 * Hashes data[0..len) and compares with expected[0..20).  The engine borrows
 * `data` until the completion carrying `tag` has been returned by vx_poll;
 * it never frees or keeps it afterwards.  Never blocks on the GPU unless every
 * slot is in flight, in which case it waits for the oldest batch (the
 * reference's spawn never refuses work either).
 *
 * Ownership rule (vx_submit and vx_submit_piece): the piece is taken iff the
 * call returns 0.  0 means exactly one completion carrying `tag` will come
 * from vx_poll, or, if the context fails later, the tag is one of the
 * vx_pending() pieces never returned (INTEGRATION.md "Device failure").  Any
 * negative return means the piece was NOT taken: no completion will ever
 * carry `tag`, and the caller hashes the piece elsewhere (vortex: the original
 * scope.spawn closure).  Per code:
 *   VX_EINVAL   NULL context or data, or (vx_submit_piece) an index outside
 *               the piece table; the context is unchanged.
 *   VX_ERANGE   len > max_piece_len; the context is unchanged.
 *   VX_ENOMEM   the pinned stage for an unregistered piece could not be
 *               allocated; the context stays usable (a later submit may
 *               succeed, e.g. from a registered buffer).
 *   VX_EDEVICE  a launch failed (this call's batch-full launch, or the launch
 *               of the previous batch) or a batch failed while this call
 *               waited for a slot.  The context is dead from now on (every
 *               call returns the code); pieces taken earlier are recovered
 *               through vx_poll as documented there.  If this call's own
 *               batch launch failed part way, the device may still read
 *               `data` until vx_destroy returns.
 *   VX_EBUSY    (only with vx_config.refuse_when_full = 1) every slot is in
 *               flight and the open batch is full: the piece was NOT taken
 *               and nothing waited; hash it on the caller's pool.  Before
 *               refusing, the call may have launched the full open batch (the
 *               launch the next submit makes anyway; stats.batches + 1) and
 *               harvested finished batches without blocking (their results
 *               wait for vx_poll).  No piece changes owner: vx_pending() is
 *               the same before and after a refused call.
 * (VX_ENODEV is not returned by submits.) */
int vx_submit(vx_ctx* ctx, uint64_t tag, const uint8_t* data, uint32_t len, const uint8_t* expected);
/* Device-resident expected-digest table: upload the
 * torrent's `pieces` string (metadata.pieces, n_pieces x 20 B, the table the
 * closure indexes at peer_connection.rs:1146) once; vx_submit_piece then
 * names a row instead of passing 20 bytes per piece.  Replaces any previous
 * table; requires no pieces in flight. */
int vx_set_piece_table(vx_ctx* ctx, const uint8_t* table, uint32_t n_pieces);
/* vx_submit with expected = row piece_index of the piece table (same
 * ownership rule and return codes, VX_EBUSY under refuse_when_full included:
 * the full open batch may be launched and finished batches harvested before
 * the refusal, the refused piece is not taken). */
int vx_submit_piece(vx_ctx* ctx, uint64_t tag, const uint8_t* data, uint32_t len, uint32_t piece_index);
/* Launch whatever is queued (call once per event-loop turn, next to the
 * drain at event_loop.rs:554-557).  If launching would leave no batch slot
 * free for the next vx_submit, the queued pieces stay open and keep
 * collecting, and the next vx_poll launches them once a batch completes:
 * under load batches grow instead of vx_submit blocking the loop thread. */
int vx_flush(vx_ctx* ctx);
/* Replaces `downloaded_piece_rc.try_recv()` (torrent.rs:418): non-blocking,
 * returns how many completions were written to out[0..max).  Order is the
 * order batches finish, which like the reference is not submission order.
 * Returns a negative VX_E* if a batch failed on the device.  After such a
 * failure the context is dead (every call returns the error), but vx_poll
 * still hands out the results of batches that did finish, and returns the
 * error only once none is left: the tags never returned are the pieces to
 * hash elsewhere (INTEGRATION.md "Device failure"), and vx_pending() is then
 * exactly their number. */
int64_t vx_poll(vx_ctx* ctx, vx_completion* out, size_t max);
/* Flush and block until every submitted piece has completed (results stay
 * queued for vx_poll).  timeout_ms = 0 waits forever. */
int vx_drain(vx_ctx* ctx, uint32_t timeout_ms);
/* Pieces submitted but not yet returned by vx_poll. */
uint64_t vx_pending(const vx_ctx* ctx);

/* ---- observability ------------------------------------------------------
 * vortex's hashing is invisible to its `metrics` feature (no
 * hash-time metric; the exported series are pieces_completed,
 * disk_write_time_ms, buffer_lifetime_ms ..., event_loop.rs:976-993,
 * buf_pool.rs:149-154).  These counters let the event loop export hash
 * throughput, mismatches, loop stalls and batch latency.  Cumulative since
 * vx_create or the last vx_reset_stats; host-side bookkeeping only (a clock
 * read per batch, none per piece).  Read them from the thread that drives the
 * context, like every other call. */
#define VX_STATS_HIST 24
typedef struct vx_stats {
    uint64_t pieces_completed;    /* results produced: async completions, host-batch and re-verified pieces */
    uint64_t pieces_mismatched;   /* of those compared with an expected digest, how many differed        */
    uint64_t bytes_completed;     /* piece bytes behind pieces_completed                                 */
    uint64_t batches;             /* whole-piece batches launched (async, host batches, re-verify slots) */
    uint64_t chunk_rounds;        /* resumable chunk rounds launched (long pieces)  */
    uint64_t gather_tiles;        /* 64 KiB tiles the gather kernel pulled from registered host buffers  */
    uint64_t staged_bytes;        /* bytes copied into pinned staging from unregistered caller memory    */
    uint64_t io_errors;           /* re-verified pieces with a failed or short read (torrent.rs:731-737) */
    uint64_t submit_stall_ns;     /* time submits waited for a batch to finish (the loop thread blocked) */
    uint64_t batch_latency_count; /* whole-piece batches harvested                                       */
    uint64_t batch_latency_sum_us; /* first submit of a batch -> its results harvested, summed           */
    uint64_t batch_latency_max_us;
    uint64_t batch_latency_hist[VX_STATS_HIST]; /* batches per [2^k, 2^(k+1)) us; [0] holds < 2 us, the last bucket everything longer */
    uint64_t zero_copy_slots;     /* (ABI 3) batches hashed straight out of registered host memory (§6.5)  */
    uint64_t zero_copy_loader_slots; /* (ABI 3) ... of them in the three-wave form (slots of < 128 pieces) */
    uint64_t submits_refused;     /* (ABI 3) async submits refused with VX_EBUSY (refuse_when_full)          */
} vx_stats;
int vx_get_stats(const vx_ctx* ctx, vx_stats* out);
int vx_reset_stats(vx_ctx* ctx);

/* Where the last vx_verify_files / _range call on ctx spent its time: the
 * startup re-verify's budget an operator sees (reads, PCIe copies, the tail).
 * Host times are steady-clock; copy times are the GPU's own (events around
 * each data H2D) and exist only on the resumable chunk path (pieces >= 2
 * chunks). */
typedef struct vx_verify_trace {
    double wall_ms;        /* the whole call                                          */
    double read_busy_ms;   /* pread time summed over the reader threads               */
    double read_span_ms;   /* first read started -> last read finished                */
    double first_read_ms;  /* call start -> first read finished (nothing overlaps it) */
    double copy_busy_ms;   /* GPU-timed data copies, summed (chunk path)              */
    double copy_span_ms;   /* first copy start -> last copy end, GPU clock            */
    double tail_ms;        /* last round enqueued -> verdicts on the host             */
    uint64_t read_bytes;   /* bytes pread                                             */
    uint64_t copy_bytes;   /* bytes of the timed copies                               */
    uint32_t readers;      /* reader threads                                          */
    uint32_t rounds;       /* timed copies (chunk rounds)                             */
    uint64_t direct_bytes; /* of read_bytes, read with O_DIRECT (not cached; §6.1)    */
    uint64_t chunk_bytes;  /* chunk of the resumable rounds (0: whole-piece slots)    */
} vx_verify_trace;
int vx_last_verify(const vx_ctx* ctx, vx_verify_trace* out);

/* The same call's round timeline (chunk path; none on the whole-piece path):
 * one record per round, in enqueue order, every time in ms from the call's
 * start on the host's steady clock.  GPU times are mapped onto it through an
 * event recorded on an idle stream at the call's start (error: that event's
 * dispatch latency, tens of us).  A gap on the copy engine between round k-1's
 * copy_end_ms and round k's copy_start_ms is the reads' when round k's
 * read_done_ms came after it, the hand-off's when its enqueue_ms did, and
 * otherwise the device's (stream dependencies). */
#define VX_ROUND_NEW_WINDOW 1u /* first round of a window of pieces              */
#define VX_ROUND_HEAD_RAMP 2u  /* a shortened round of the call's first chunk     */
#define VX_ROUND_TAIL_RAMP 4u  /* a shortened round of the call's last chunk      */
typedef struct vx_verify_round {
    double read_submit_ms; /* its reads queued on the reader pool                 */
    double read_done_ms;   /* its last read finished                              */
    double enqueue_ms;     /* its data copy and chunk kernel enqueued              */
    double copy_start_ms;  /* GPU: its data copy began (0 when not timed)         */
    double copy_end_ms;    /* GPU: its data copy ended                            */
    double kernel_end_ms;  /* GPU: its chunk kernel ended                         */
    uint64_t bytes;        /* bytes copied                                        */
    uint64_t offset;       /* the chunk's offset inside its pieces                */
    uint32_t lanes;        /* pieces in the round                                 */
    uint32_t flags;        /* VX_ROUND_*                                          */
} vx_verify_round;
/* Writes up to max records to out (may be NULL with max 0) and returns how
 * many rounds the call had. */
int64_t vx_last_verify_rounds(const vx_ctx* ctx, vx_verify_round* out, size_t max);

/* ---- synchronous host batches (bulk re-verify, torrent.rs:724-740) ----- */
/* digests_out: n*20 bytes.  Pieces are pipelined through the slots, longest
 * first (ragged batches: DESIGN.md §6.4); outputs are always in the caller's
 * order.  Pieces may be of any lengths up to max_piece_len. */
int vx_sha1_batch(vx_ctx* ctx, const uint8_t* const* ptrs, const uint32_t* lens, size_t n, uint8_t* digests_out);
/* expected: n*20 bytes; matched_out: n bytes of 0/1 (the Box<[bool]> of
 * torrent.rs:727-740); digests_out may be NULL. */
int vx_verify_batch(vx_ctx* ctx, const uint8_t* const* ptrs, const uint32_t* lens, const uint8_t* expected,
                    size_t n, uint8_t* matched_out, uint8_t* digests_out);

/* ---- bulk re-verify from disk (torrent.rs:716-761, file_store.rs:228-303)
 * The torrent's files in order (path, length); the layout follows
 * FileStore::new (file_store.rs:126-160): pieces run across file boundaries,
 * piece i has piece_length bytes except the last (piece_selector.rs:63-69).
 * Every piece's segments are pread (io_threads readers, 0 = default) into
 * pinned batch buffers that stream to the GPU while the next batch is read.
 * matched_out[i] = 1 iff piece i was read completely and its SHA-1 equals
 * expected[20*i..].  A piece whose file is missing, short or unreadable is
 * matched = 0, like the reference's `Err(_) => false` (torrent.rs:731-737).
 * Returns the number of pieces that hit an I/O error (>= 0) or a VX_E* code.
 * Requires no async pieces pending on ctx. */
int64_t vx_verify_files(vx_ctx* ctx, const char* const* paths, const uint64_t* file_lengths, size_t nfiles,
                        uint32_t piece_length, const uint8_t* expected, size_t n_pieces, uint8_t* matched_out,
                        uint32_t io_threads);
/* Pieces [first, first+count) of the same torrent only: one rank's shard of a
 * multi-GPU re-verify (python: vortex_amd.shard.verify_files_sharded).
 * expected is still the whole n_pieces*20 table; matched_out has count
 * bytes, matched_out[k] for piece first+k.  Only that range's bytes are read.
 * vx_verify_files(...) is vx_verify_files_range(..., 0, n_pieces, ...). */
int64_t vx_verify_files_range(vx_ctx* ctx, const char* const* paths, const uint64_t* file_lengths, size_t nfiles,
                              uint32_t piece_length, const uint8_t* expected, size_t n_pieces, size_t first,
                              size_t count, uint8_t* matched_out, uint32_t io_threads);
/* ---- the self-balancing split (round 6) ---------------
 * One bulk re-verify shared at once by the engine and the caller's own pool
 * with no plan: torrent.rs:724-740's par_iter balances by rayon work
 * stealing, and this does the same across the PCIe boundary.  A vx_split is
 * one claim word over pieces [first, end): the pool takes pieces one by one
 * from the head (vx_split_claim, one compare-and-swap each), the engine takes
 * whole groups from the top as it forms its chunk rounds, and the two meet
 * wherever the host at hand puts them.  Before every round the engine
 * compares its remaining time with the pool's, both from rates measured in
 * this call (the pool's finished pieces per second through vx_split_done;
 * its own copy, read and per-block chain rates from the rounds' GPU events),
 * and takes the group of pieces that keeps the two finish times equal.
 * Its first group, before anything is measured, comes from the previous
 * split calls on the same context (their rates, and how far their finish
 * times strayed from the prediction), else from cpu_threads x
 * cpu_thread_rate and the PCIe rate.  The caller owns the struct; it may live
 * on the stack of the thread that starts both sides. */
typedef struct vx_split {
    uint64_t word;          /* head (low 32 bits) | stop (high 32): [head, stop) is unclaimed          */
    uint64_t pool_done;     /* pieces the pool finished (vx_split_done)                                */
    uint64_t start_ns;      /* steady clock at vx_split_init: the pool's rate is measured from here     */
    uint64_t first;         /* the range [first, end)                                                  */
    uint64_t end;
    uint32_t cpu_threads;   /* the pool's threads (0 = no pool: the engine takes every piece)          */
    uint32_t engines;       /* engines claiming at once (0 or 1: one; vx_verify_files_split_multi sets it) */
    double cpu_thread_rate; /* the pool's bytes/s per thread alone (cold start only; 0 = 2.2e9, SHA-NI) */
    uint64_t pool_last_ns;  /* steady clock at the pool's latest vx_split_done (when the pool finished)  */
} vx_split;
/* Pieces [first, end) unclaimed; end - first < 2^32 and end < 2^32. */
int vx_split_init(vx_split* s, uint64_t first, uint64_t end, uint32_t cpu_threads, double cpu_thread_rate);
/* Pool side, from any number of threads: the next piece from the head, or -1
 * when no piece is left for the pool.  After a piece's verdict is written,
 * call vx_split_done(s, 1): the engine reads the pool's rate from it. */
int64_t vx_split_claim(vx_split* s);
void vx_split_done(vx_split* s, uint64_t pieces);
/* The lowest piece the engine took (end when it took none): once both sides
 * have returned, the pool verified [first, boundary) and the engine
 * [boundary, end). */
uint64_t vx_split_boundary(const vx_split* s);
/* The engine's side: verifies the pieces it claims from s (always the top of
 * the range, contiguous) with resumable chunk rounds, while the caller's pool
 * runs vx_split_claim on its own threads; returns when its pieces are done.
 * If the pool has reported verdicts and is still working then, the engine
 * waits for it (polling, at most 3x its estimated remaining time + 50 ms) to
 * learn how far the two finish times strayed, for the next call's first
 * group; a pool that has reported nothing yet is not waited for, so a caller
 * may also run its pool after this returns.  With nothing in flight, the
 * engine takes the unclaimed pieces itself when the pool has finished none
 * for a while (two of its piece times, at least 4 ms): a pool busy elsewhere
 * does not leave them waiting.  matched_out has end - first bytes
 * (matched_out[k] for piece first + k); the engine writes only its own
 * pieces' entries, the pool writes the others.  Returns the number of the
 * engine's pieces that hit an I/O error (>= 0), or a VX_E* code: then the
 * pieces [vx_split_boundary(s), end) have no verdict and the caller verifies
 * them itself.  A split declared for one engine (engines 0 or 1) refuses a
 * second one with VX_EINVAL; with engines = k, k calls on k contexts may
 * claim from it at once (each engine's pieces are then its own groups, not
 * one tail).  Requires no async pieces pending on ctx.  vx_last_verify and
 * vx_last_verify_rounds describe the call as for vx_verify_files. */
int64_t vx_verify_files_split(vx_ctx* ctx, const char* const* paths, const uint64_t* file_lengths, size_t nfiles,
                              uint32_t piece_length, const uint8_t* expected, size_t n_pieces, vx_split* s,
                              uint8_t* matched_out, uint32_t io_threads);
/* The split over several GPUs of one process (one context per GPU, as for
 * vx_verify_files_multi) and the caller's pool at once: sets s->engines =
 * nctx and runs vx_verify_files_split on every context on its own host
 * thread, io_threads (the total) divided among them.  Returns the summed I/O
 * errors of the engines' pieces, or the first failing context's VX_E* code
 * (then re-verify [vx_split_boundary(s), end) on the pool: some of it has
 * verdicts, not all). */
int64_t vx_verify_files_split_multi(vx_ctx* const* ctxs, size_t nctx, const char* const* paths,
                                    const uint64_t* file_lengths, size_t nfiles, uint32_t piece_length,
                                    const uint8_t* expected, size_t n_pieces, vx_split* s, uint8_t* matched_out,
                                    uint32_t io_threads);
/* In-process multi-GPU re-verify: vortex is one process with one event loop
 * (event_loop.rs:385), so on a multi-GPU host it holds one context per GPU
 * (vx_config.device) and hands them all to this call, which replaces the
 * whole par_iter of torrent.rs:724-740.  Pieces [0, n_pieces) are split into
 * nctx contiguous ranges (n_pieces/nctx each, the remainder to the last
 * contexts — the rule of vortex_amd.shard.shard_range) and context k verifies
 * range k on its own host thread with vx_verify_files_range, writing
 * matched_out[first_k ..] in place.  io_threads is the total reader count,
 * divided among the contexts (0 = default).  Contexts must be distinct and
 * idle; they may share a device.  Returns the summed I/O-error count, or the
 * first failing context's VX_E* code (vx_last_error names the context). */
int64_t vx_verify_files_multi(vx_ctx* const* ctxs, size_t nctx, const char* const* paths,
                              const uint64_t* file_lengths, size_t nfiles, uint32_t piece_length,
                              const uint8_t* expected, size_t n_pieces, uint8_t* matched_out, uint32_t io_threads);

/* ---- planning: where should a bulk verify run? (host-only, no GPU) -----
 * One piece is one lane on the GPU and SHA-1 cannot be split inside a
 * piece, so a few very long pieces are bound by one lane's chain (~0.76 us
 * per 64-byte block, ~84 MB/s), while vortex's own rayon + `sha1` pool
 * (torrent.rs:724-740) hashes one piece per core at ~2 GB/s.  This cost model
 * (calibrated on MI355X) predicts both for n_pieces pieces of
 * piece_length bytes (total_length in all, the last piece shorter) read from
 * host memory or the page cache, so the caller can keep its own pool where it
 * is faster (INTEGRATION.md "Where the GPU pays").  cpu_threads / cpu_thread_rate
 * describe the caller's pool (0 = 16 threads / 2.2e9 B/s per thread, SHA-NI). */
typedef struct vx_plan {
    double gpu_s;               /* predicted e2e seconds of vx_verify_files / vx_verify_batch   */
    double gpu_chain_s;         /* one piece's chain of compressions in one lane               */
    double gpu_transfer_s;      /* all bytes over PCIe                                         */
    double cpu_s;               /* predicted seconds of the caller's pool                      */
    double piece_latency_s;     /* download path: submit-to-poll floor of one piece on the GPU */
    double cpu_piece_latency_s; /* the same piece on one pool thread                           */
    int32_t use_gpu;            /* 1 when 1.1 * gpu_s < cpu_s (near a tie, keep the CPU pool)  */
    uint32_t _pad;
} vx_plan;
int vx_plan_verify(uint64_t n_pieces, uint32_t piece_length, uint64_t total_length, uint32_t cpu_threads,
                   double cpu_thread_rate, vx_plan* out);
/* The same plan for a verify split over n_gpus contexts, one per GPU
 * (vx_verify_files_multi): gpu_transfer_s is each GPU's share over its own
 * link; gpu_chain_s, one piece's chain, does not shrink with more GPUs.
 * n_gpus 0 or 1 gives vx_plan_verify's answer. */
int vx_plan_verify_gpus(uint64_t n_pieces, uint32_t piece_length, uint64_t total_length, uint32_t cpu_threads,
                        double cpu_thread_rate, uint32_t n_gpus, vx_plan* out);
/* Split one bulk verify between the GPUs and the caller's own pool, both
 * running at once (torrent.rs:724-740's par_iter over the pool's range, and
 * vx_verify_files_range / _multi over the GPUs' range): the GPUs take the
 * contiguous tail [*gpu_first, n_pieces), *gpu_count pieces, chosen so the
 * predicted GPU time (the same model over n_gpus, its bytes at 0.74 of the
 * link: the pool shares host memory) meets the pool's time on the rest (at
 * 0.80 of cpu_thread_rate: the engine's readers share it too).
 * cpu_threads is the pool that runs beside the engine: leave the engine's
 * readers their cores (e.g. 12 pool threads beside 8 readers on 16 cores;
 * INTEGRATION.md "The split").  *gpu_count is 0 when no split beats the pool
 * alone by the 10 % margin, and n_pieces when the GPUs alone are fastest.
 * out (may be NULL) gets the plan of the split: gpu_s for the GPUs' range,
 * cpu_s for the pool's, use_gpu = 1 when the GPUs take part. */
int vx_plan_verify_split(uint64_t n_pieces, uint32_t piece_length, uint64_t total_length, uint32_t cpu_threads,
                         double cpu_thread_rate, uint32_t n_gpus, uint64_t* gpu_first, uint64_t* gpu_count,
                         vx_plan* out);

/* ---- device-resident batches (the hot path; no context needed) --------
 * These entries validate what they can see on the host — NULL pointers, the
 * alignment of d_base and stride, stride >= len — and nothing that lives in
 * device memory: d_offsets, d_lens and d_order are read only by the kernel,
 * so a misaligned or out-of-range offset, a length running past the
 * allocation or an order index >= n is NOT detected here and makes the
 * kernel read (or fault on) memory outside the batch.  Callers that build
 * the layout on the host check it there; the Python wrapper
 * vortex_amd.device.sha1_ragged checks it on the device before launching. */
/* Pieces i in [0,n) at d_base + i*stride, each len bytes.  Writes
 * d_digests[20*i..] (may be NULL) and, when d_expected is given,
 * d_matched[i] = (digest == d_expected[20*i..]) (0/1).  stride and d_base
 * must be multiples of 16 and stride >= len. */
int vx_sha1_device_uniform(const void* d_base, uint64_t stride, uint32_t len, uint32_t n, void* d_digests,
                           const void* d_expected, void* d_matched, void* stream);
/* Ragged batch: piece i at d_base + d_offsets[i] (16-byte aligned), d_lens[i]
 * bytes.  d_order (may be NULL) is a permutation of [0,n) telling lane j to
 * hash piece d_order[j]; pass pieces sorted by descending length so each
 * wavefront gets equal-length work (see vx_sort_order).  Runs the kernel
 * suited to chain-bound batches (lengths that differ). */
int vx_sha1_device_ragged(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lens,
                          const uint32_t* d_order, uint32_t n, void* d_digests, const void* d_expected,
                          void* d_matched, void* stream);
/* As vx_sha1_device_ragged, with the batch's longest piece and total bytes
 * (known on the host when the batch is laid out) so the engine picks the
 * kernel whose time bound, throughput or longest chain, is lower. */
int vx_sha1_device_ragged_hint(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lens,
                               const uint32_t* d_order, uint32_t n, uint32_t max_len, uint64_t total_len,
                               void* d_digests, const void* d_expected, void* d_matched, void* stream);
/* Host helper: write into order_out the permutation that sorts lens[0..n)
 * by descending length (stable).  Used to build d_order. */
int vx_sort_order(const uint32_t* lens, uint32_t n, uint32_t* order_out);

#ifdef __cplusplus
}
#endif
#endif /* VX_HASH_H */
