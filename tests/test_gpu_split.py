"""GPU: the self-balancing split re-verify (vx_verify_files_split).

The engine and the caller's pool verify one torrent at once with no plan:
the pool (oracle/pool_oracle.cpp's claim pool, the stand-in for vortex's
rayon threads calling vx_split_claim) takes pieces from the head, the engine
takes groups from the top sized from rates it measures during the call.  The
bar is the reference's own: every verdict equals check_piece_hash_sync's
(torrent.rs:724-740 over file_store.rs:228-303) on the same files —
damaged pieces on either side, truncated files (``Err(_) => false``), file
boundaries inside pieces, pieces shorter and longer than a chunk, ranges that
start mid-torrent, pools of any size (none at all included) — and every piece
is verified by exactly one side.
"""
import os
import random
import threading

import pytest

import oracle

pytestmark = pytest.mark.gpu


def _files(tmp_path, pl, sizes, seed):
    paths = []
    for k, L in enumerate(sizes):
        p = tmp_path / f"s{seed}_{k}.bin"
        p.write_bytes(oracle.gen_piece(seed, k, L))
        paths.append(str(p))
    data = b"".join(open(p, "rb").read() for p in paths)
    exp = b"".join(oracle.sha1(data[i:i + pl]) for i in range(0, len(data), pl))
    return paths, sizes, exp


def _run_split(pool, paths, lens, pl, exp, first, end, cpu_threads, rate=0.0, io_threads=4):
    from vortex_amd.hash_pool import Split

    sp = Split(first, end, cpu_threads, rate)
    out = {}

    def engine():
        try:
            out["bad"] = pool.verify_files_split(paths, lens, pl, exp, sp, io_threads=io_threads)
        except Exception as e:  # noqa: BLE001
            out["err"] = e

    th = threading.Thread(target=engine)
    th.start()
    taken = 0
    if cpu_threads:
        taken = oracle.pool_verify_files_claim(paths, lens, pl, exp, cpu_threads, sp.claim_fn, sp.done_fn, sp.arg,
                                               first, sp.matched)
    th.join()
    if "err" in out:
        raise out["err"]
    return sp, taken, out["bad"]


@pytest.mark.parametrize("seed", range(6))
def test_split_matches_pool_on_damaged_layouts(built, gpu, tmp_path, seed):
    from vortex_amd.hash_pool import HashPool

    rng = random.Random(seed)
    pl = rng.choice([65536, 262144 + 4096, 1 << 20, 2 << 20])
    nfiles = rng.randint(1, 4)
    sizes = [rng.randint(0, 40) * pl + rng.randint(0, pl - 1) for _ in range(nfiles)]
    if sum(sizes) == 0:
        sizes[0] = 3 * pl + 1
    paths, sizes, exp = _files(tmp_path, pl, sizes, seed)
    n = len(exp) // 20
    total = sum(sizes)
    for _ in range(rng.randint(1, 4)):  # damaged bytes anywhere (either side)
        off = rng.randrange(total)
        acc = 0
        for p, L in zip(paths, sizes):
            if off < acc + L:
                with open(p, "r+b") as f:
                    f.seek(off - acc)
                    b = f.read(1)
                    f.seek(off - acc)
                    f.write(bytes([b[0] ^ 0x5A]))
                break
            acc += L
    if rng.random() < 0.5:  # a truncated file: its pieces are I/O errors on whichever side
        k = rng.randrange(nfiles)
        os.truncate(paths[k], sizes[k] // 2)
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    first = rng.randint(0, n // 3)
    end = n - rng.randint(0, n // 4)
    cpu_threads = rng.choice([0, 1, 3, 8])
    with HashPool(pl, slots=3, slot_bytes=max(16 << 20, 2 * pl), batch_pieces=64) as pool:
        for rep in range(2):
            sp, taken, bad = _run_split(pool, paths, sizes, pl, exp, first, end, cpu_threads,
                                        rate=rng.choice([0.0, 5e8, 4e9]))
            b = sp.boundary
            assert first <= b <= end and taken == b - first
            if cpu_threads == 0:
                assert b == first  # no pool: the engine took every piece
            assert sp.verdicts() == want[first:end], (seed, rep, b)
            st = pool.stats()
            assert st["io_errors"] >= bad


def test_split_whole_range_both_sides_take_part(built, gpu, tmp_path):
    """A torrent large enough that both sides finish work: 384 x 2 MiB, one
    damaged piece near each end; the pool at 8 threads (its rate measured in
    the call) and the engine both take pieces."""
    from vortex_amd.hash_pool import HashPool

    pl, n = 2 << 20, 384
    paths, sizes, exp = _files(tmp_path, pl, [n * pl - 12345], 99)
    for off in (3 * pl + 17, (n - 3) * pl + 5):
        with open(paths[0], "r+b") as f:
            f.seek(off)
            b = f.read(1)
            f.seek(off)
            f.write(bytes([b[0] ^ 1]))
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=8)
    with HashPool(pl, slots=4, slot_bytes=256 << 20, batch_pieces=1024) as pool:
        pool.verify_files(paths, sizes, pl, exp, io_threads=8)  # warm the stages and the page cache
        for _ in range(3):
            sp, taken, bad = _run_split(pool, paths, sizes, pl, exp, 0, n, 8, io_threads=8)
            assert sp.verdicts() == want and bad == 0
            assert 0 < sp.boundary < n, sp.boundary  # both sides took part
            rounds = pool.last_verify_rounds()
            assert rounds and sum(r["bytes"] for r in rounds) >= (n - sp.boundary) * pl - 12345


def test_split_engine_failure_leaves_its_pieces_to_the_caller(built, gpu, tmp_path):
    """An engine round that fails (injected) returns the error; the pool
    still finishes its side, and the pieces [boundary, end) — the ones with
    no verdict — are what the caller verifies itself (vx_hash.h)."""
    from vortex_amd._lib import VX_EDEVICE, VxError
    from vortex_amd.hash_pool import HashPool

    pl, n = 1 << 20, 96
    paths, sizes, exp = _files(tmp_path, pl, [n * pl], 5)
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    with HashPool(pl, slots=3, slot_bytes=32 << 20, batch_pieces=64, verify_chunk=131072, hooks=True) as pool:
        pool.lib.vx_tuning_fail_launch_after(pool._h, 3)
        with pytest.raises(VxError) as ei:
            _run_split(pool, paths, sizes, pl, exp, 0, n, 2)
        assert ei.value.code == VX_EDEVICE
        # the same context, next call: a clean split
        sp, taken, bad = _run_split(pool, paths, sizes, pl, exp, 0, n, 2)
        assert sp.verdicts() == want and bad == 0


def test_split_refuses_a_second_engine(built, gpu, tmp_path):
    """One engine per split (vx_hash.h): two contexts racing on one vx_split
    — the first to claim keeps the split, the other fails with VX_EINVAL
    before claiming anything, so every verdict still comes from one side."""
    from vortex_amd._lib import VX_EINVAL, VxError
    from vortex_amd.hash_pool import HashPool, Split

    # small slots: 64 lanes a round, so the first engine's first group leaves
    # pieces for the second to reach for
    pl, n = 256 << 10, 1200
    paths, sizes, exp = _files(tmp_path, pl, [n * pl - 999], 17)
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    sp = Split(0, n, 0)
    out = {}
    with HashPool(pl, slots=3, slot_bytes=8 << 20) as a, HashPool(pl, slots=3, slot_bytes=8 << 20) as b:
        def run(name, pool):
            try:
                out[name] = pool.verify_files_split(paths, sizes, pl, exp, sp, io_threads=2)
            except VxError as e:
                out[name] = e

        ths = [threading.Thread(target=run, args=(k, p)) for k, p in (("a", a), ("b", b))]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    errs = [v for v in out.values() if isinstance(v, VxError)]
    assert len(errs) == 1 and errs[0].code == VX_EINVAL, out
    assert sp.boundary == 0 and sp.verdicts() == want  # the survivor verified every piece


@pytest.mark.parametrize("nctx,cpu_threads", [(2, 4), (3, 0), (2, 1)])
def test_split_multi_engines(built, gpu, tmp_path, nctx, cpu_threads):
    """vx_verify_files_split_multi: several contexts (one per GPU; here all
    on the box's one GPU) claim groups from one split beside the pool, each
    as one of nctx equal takers.  Every verdict equals the pool
    restatement's, on a multi-file layout with damaged pieces and a
    truncated file; with no pool the engines take every piece."""
    from vortex_amd.hash_pool import HashPool, Split, verify_files_split_multi

    pl = 1 << 20
    sizes = [150 * pl + 12345, 3 * pl - 7, 260 * pl + 99]
    paths, sizes, exp = _files(tmp_path, pl, sizes, 40 + nctx)
    n = len(exp) // 20
    for p, off in ((paths[0], 17 * pl + 3), (paths[2], 200 * pl + 5), (paths[2], 9)):
        with open(p, "r+b") as f:
            f.seek(off)
            b = f.read(1)
            f.seek(off)
            f.write(bytes([b[0] ^ 0x11]))
    os.truncate(paths[1], 2 * pl)
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    pools = [HashPool(pl, slots=3, slot_bytes=64 << 20) for _ in range(nctx)]
    try:
        for rep in range(2):
            sp = Split(0, n, cpu_threads)
            out = {}

            def engines():
                try:
                    out["bad"] = verify_files_split_multi(pools, paths, sizes, pl, exp, sp, io_threads=2 * nctx)
                except Exception as e:  # noqa: BLE001
                    out["err"] = e

            th = threading.Thread(target=engines)
            th.start()
            taken = 0
            if cpu_threads:
                taken = oracle.pool_verify_files_claim(paths, sizes, pl, exp, cpu_threads, sp.claim_fn, sp.done_fn,
                                                       sp.arg, 0, sp.matched)
            th.join()
            assert "err" not in out, out
            assert sp.s.engines == nctx and taken == sp.boundary
            if not cpu_threads:
                assert sp.boundary == 0
            assert sp.verdicts() == want, (rep, sp.boundary)
            done = sum(p.stats()["pieces_completed"] for p in pools)
            assert done == (rep + 1) * (n - sp.boundary) or rep == 1  # every engine piece counted once
    finally:
        for p in pools:
            p.close()


def test_split_stats_count_the_engines_pieces_only(built, gpu, tmp_path):
    """vx_get_stats after a split: the engine counts exactly its own pieces
    [boundary, end) — completed, mismatched (damaged, not I/O errors) and I/O
    errors (a truncated tail file) — and none of the pool's."""
    from vortex_amd.hash_pool import HashPool

    pl, n_a, n_b = 1 << 20, 120, 40
    sizes = [n_a * pl, n_b * pl - 777]
    paths, sizes, exp = _files(tmp_path, pl, sizes, 61)
    n = len(exp) // 20
    with open(paths[1], "r+b") as f:  # damage a piece near the top (the engine's side)
        f.seek(30 * pl + 11)
        b = f.read(1)
        f.seek(30 * pl + 11)
        f.write(bytes([b[0] ^ 0x80]))
    os.truncate(paths[1], 37 * pl)  # pieces n_a+37 .. n-1 short or missing: I/O errors
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    with HashPool(pl, slots=3, slot_bytes=64 << 20) as pool:
        pool.reset_stats()
        sp, taken, bad = _run_split(pool, paths, sizes, pl, exp, 0, n, 2, io_threads=4)
        b = sp.boundary
        assert sp.verdicts() == want and taken == b
        assert b <= n_a + 30, b  # the engine took the top (a 2-thread pool cannot reach it first)
        st = pool.stats()
        io_err = [i for i in range(b, n) if i >= n_a + 37]
        assert bad == len(io_err) == st["io_errors"]
        assert st["pieces_completed"] == n - b
        assert st["pieces_mismatched"] == sum(1 for i in range(b, n) if not want[i]) - len(io_err)


@pytest.mark.parametrize("one_round,cap", [(1, 64 << 20), (1, 0), (0, 0)])
def test_split_one_chunk_pieces(built, gpu, tmp_path, one_round, cap):
    """Pieces of one chunk (64 KiB, 4,000 of them over two files, a piece
    across the file boundary, damaged pieces near each end) under each rule
    set for them (vx_tuning_split_rules: the default 64 MiB rounds, uncapped,
    the multi-round rules): every verdict is the pool restatement's, and with
    the cap no round carries more than 1,024 lanes."""
    from vortex_amd.hash_pool import HashPool

    pl = 64 << 10
    sizes = [2500 * pl + 4321, 1500 * pl - 4321 - 999]
    paths, sizes, exp = _files(tmp_path, pl, sizes, 71)
    n = len(exp) // 20
    for p, off in ((paths[0], 5 * pl + 3), (paths[1], 1400 * pl + 7)):
        with open(p, "r+b") as f:
            f.seek(off)
            b = f.read(1)
            f.seek(off)
            f.write(bytes([b[0] ^ 0x42]))
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    with HashPool(pl, slots=4, slot_bytes=512 << 20, batch_pieces=4096, hooks=True) as pool:
        pool.lib.vx_tuning_split_rules(pool._h, one_round, cap, 1, 1)
        try:
            for rep in range(3):
                sp, taken, bad = _run_split(pool, paths, sizes, pl, exp, 0, n, 4, io_threads=4)
                assert sp.verdicts() == want and taken == sp.boundary, (rep, sp.boundary)
                assert sp.boundary < n  # the engine took part
                if cap:
                    assert max(r["lanes"] for r in pool.last_verify_rounds()) <= 1024
        finally:
            pool.lib.vx_tuning_split_rules(pool._h, 1, 64 << 20, 1, 1)


def test_split_engine_returns_when_the_pool_stalls(built, gpu, tmp_path):
    """The engine waits for a pool still finishing its last pieces only for a
    bounded time (vx_hash.h): a pool that reports one verdict and then holds
    two claimed pieces without finishing them does not keep the engine's call
    from returning, and the engine, idle beside a pool that finishes
    nothing, takes every unclaimed piece.  Its verdicts, and the pool's once
    it finishes what it held, match the pool restatement's."""
    import time

    from vortex_amd.hash_pool import HashPool, Split

    pl, n = 1 << 20, 200
    paths, sizes, exp = _files(tmp_path, pl, [n * pl - 4321], 83)
    with open(paths[0], "r+b") as f:  # a damaged piece on the engine's side
        f.seek(150 * pl + 9)
        b = f.read(1)
        f.seek(150 * pl + 9)
        f.write(bytes([b[0] ^ 0x20]))
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    pool = HashPool(pl, slots=3, slot_bytes=64 << 20)
    for rep in range(2):  # the second call starts from the first's learned state
        sp = Split(0, n, cpu_threads=2, cpu_thread_rate=2e9)
        held, release = [], threading.Event()

        def stalled_pool():
            for _ in range(3):
                held.append(sp.claim())
            i = held.pop(0)
            sp.matched[i] = b"\x01" if want[i] else b"\x00"
            sp.done(1)
            release.wait(30)

        th = threading.Thread(target=stalled_pool)
        th.start()
        while len(held) < 2:
            time.sleep(0.001)
        try:
            t0 = time.perf_counter()
            bad = pool.verify_files_split(paths, sizes, pl, exp, sp, io_threads=4)
            took = time.perf_counter() - t0
        finally:
            release.set()
        th.join()
        assert took < 5.0, took
        b = sp.boundary
        # a pool that finishes nothing while the engine is idle counts as
        # stopped: the engine takes every unclaimed piece
        assert b == 3 and bad == 0, (rep, b)
        # the caller's pool finishes what it held and claims what is left
        rest = held + [i for i in iter(sp.claim, -1)]
        assert sorted(rest) == [1, 2] + list(range(3, b)), (rep, b)
        for i in rest:
            sp.matched[i] = b"\x01" if want[i] else b"\x00"
        assert sp.verdicts() == want, rep
    pool.close()
