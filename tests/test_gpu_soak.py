"""Bounded randomized soaks of round 5's engine paths (-m gpu, ~10 s each).

* The async download path with vx_config.refuse_when_full on and off:
  random piece lengths (empty to the pool's piece length), pieces in
  registered pool buffers and in plain memory, planted mismatches, random
  flush / poll cadence.  A refused submit (VX_EBUSY) is hashed by the test
  itself, as vortex's pool would; every piece must come back exactly once
  with hashlib's verdict, and the engine's counters must agree.
* The re-verify of random multi-file torrents (damaged, truncated and
  missing files) through the chunk rounds' copy stream, whole, split with the
  CPU pool restatement at random points (bench.split_call) and balanced at run
  time (bench.balanced_call, vx_verify_files_split): every verdict
  equals oracle.pool_verify_files (file_store.rs:228-303 restated), and every
  chunk round's timeline is ordered.
"""
import hashlib
import mmap
import os
import random
import sys
import time

import pytest

import oracle
from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("refuse", [0, 1])
def test_soak_async(built, gpu, refuse):
    from vortex_amd._lib import VX_EBUSY, VxError
    from vortex_amd.hash_pool import HashPool

    rng = random.Random(500 + refuse)
    t_end = time.time() + 8
    pools = refusals = pieces = 0
    while time.time() < t_end:
        plen = rng.choice([16384, 262144, 1 << 20, 3 << 20])
        nbuf = rng.randint(8, 48)
        with HashPool(plen, slots=rng.choice([2, 3, 4]), batch_pieces=rng.choice([4, 16, 64]),
                      refuse_when_full=refuse) as pool:
            pools += 1
            bufs = [mmap.mmap(-1, plen) for _ in range(nbuf)]
            for b in bufs:
                pool.register_buffer(b)
            inflight, verdicts, truth = {}, {}, {}
            n_bad = n_bytes = 0
            for tag in range(rng.randint(50, 300)):
                L = rng.choice([0, 1, 55, 64, plen, plen, rng.randint(1, plen)])
                body = oracle.gen_piece(77, tag, L)
                buf = bufs[tag % nbuf]
                if rng.random() < 0.3 or any(v is buf for v in inflight.values()):
                    buf = bytearray(body)  # plain memory, or that pool buffer is still in flight
                else:
                    buf[:L] = body
                good = hashlib.sha1(body).digest()
                exp = good if rng.random() > 0.05 else bytes(20)
                truth[tag] = exp == good
                try:
                    pool.spawn(tag, 3, buf, L, exp)
                    inflight[tag] = buf
                    n_bad += exp != good
                    n_bytes += L
                except VxError as e:
                    assert refuse and e.code == VX_EBUSY and e.refused[0] == tag and e.refused[2] is buf
                    refusals += 1
                    verdicts[tag] = hashlib.sha1(bytes(buf[:L])).digest() == exp  # the caller's own pool
                r = rng.random()
                if r < 0.2:
                    pool.flush()
                if r < 0.5:
                    for d in pool.try_iter():
                        assert d.index not in verdicts and d.conn_id == 3
                        verdicts[d.index] = d.hash_matched
                        inflight.pop(d.index)
            pool.drain()
            for d in pool.try_iter():
                assert d.index not in verdicts
                verdicts[d.index] = d.hash_matched
                inflight.pop(d.index)
            assert not inflight and pool.pending == 0
            assert verdicts == truth
            st = pool.stats()
            taken = len(truth) - st["submits_refused"]
            assert st["pieces_completed"] == taken and st["pieces_mismatched"] == n_bad
            assert st["bytes_completed"] == n_bytes
            if not refuse:
                assert st["submits_refused"] == 0
            pieces += len(truth)
            for b in bufs:
                pool.unregister_buffer(b)
    assert pools >= 3 and pieces > 500
    if refuse:
        assert refusals > 0, "no submit was ever refused: the soak never filled the pipeline"


def _torrent(tmp, rng, pl, k):
    sizes = [rng.choice([0, 1, 3, pl - 1, pl, pl + 5, rng.randint(1, 5 * pl)]) for _ in range(rng.randint(1, 7))]
    if sum(sizes) == 0:
        sizes[0] = pl + 7
    paths = []
    for i, L in enumerate(sizes):
        p = os.path.join(tmp, f"t{k}_{i}.bin")
        with open(p, "wb") as f:
            f.write(oracle.gen_piece(900 + k, i, L))
        paths.append(p)
    data = b"".join(open(p, "rb").read() for p in paths)
    exp = b"".join(hashlib.sha1(data[i:i + pl]).digest() for i in range(0, len(data), pl))
    # damage: a flipped byte, a truncated file, a missing file
    for p in paths:
        r = rng.random()
        size = os.path.getsize(p)
        if r < 0.15 and size:
            with open(p, "r+b") as f:
                f.seek(rng.randrange(size))
                b = f.read(1)
                f.seek(f.tell() - 1)
                f.write(bytes([b[0] ^ 1]))
        elif r < 0.22:
            os.truncate(p, size // 2)
        elif r < 0.27:
            os.unlink(p)
    return paths, sizes, exp


def test_soak_reverify_and_split(built, gpu, tmp_path):
    sys.path.insert(0, ROOT)
    import bench
    from vortex_amd.hash_pool import HashPool

    rng = random.Random(5)
    t_end = time.time() + 10
    torrents = 0
    while time.time() < t_end:
        pl = rng.choice([256 * 1024, 1 << 20, 2 << 20])  # whole-piece slots / chunk rounds on the copy stream
        d = tmp_path / f"d{torrents}"
        d.mkdir()
        paths, sizes, exp = _torrent(str(d), rng, pl, torrents)
        n = len(exp) // 20
        want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
        with HashPool(pl, slots=rng.choice([2, 3, 4]), slot_bytes=rng.choice([3, 8, 32]) << 20) as pool:
            got, bad = pool.verify_files(paths, sizes, pl, exp, io_threads=rng.choice([1, 3, 8]))
            assert got == want, (sizes, pl)
            rounds = pool.last_verify_rounds()
            for a, b in zip(rounds, rounds[1:]):
                assert b["copy_start_ms"] >= a["copy_end_ms"] - 1e-3 and b["enqueue_ms"] >= a["enqueue_ms"]
            first = rng.randint(0, n)
            r = bench.split_call(pool, paths, sizes, n, pl, exp, first, rng.choice([2, 4]), rng.choice([2, 4]))
            assert r["matched"] == want, (sizes, pl, first)
            # the self-balancing split, pool of any size and any claimed rate
            b = bench.balanced_call(pool, paths, sizes, n, pl, exp, rng.choice([1, 2, 4]), rng.choice([1, 2, 4, 8]),
                                    rng.choice([0.0, 3e8, 2e9, 2e10]))
            assert b["matched"] == want and 0 <= b["boundary"] <= n, (sizes, pl, b["boundary"])
        torrents += 1
    assert torrents >= 5


def test_soak_split_engines(built, gpu, tmp_path):
    """The balanced split on random torrents (damaged, truncated and missing
    files), random ranges, pools of 0-8 threads at any claimed rate, 1-3
    engines on one split (vx_verify_files_split_multi), random slot sizes and,
    now and then, an engine round that fails (injected): every verdict of a
    clean call equals oracle.pool_verify_files; a failed call leaves the
    context usable and its pieces [boundary, end) to the caller, who verifies
    them with the oracle.  VX_SOAK_SECONDS (default 10) sets the budget."""
    import threading

    from vortex_amd._lib import VxError
    from vortex_amd.hash_pool import HashPool, Split, verify_files_split_multi

    rng = random.Random(77)
    t_end = time.time() + float(os.environ.get("VX_SOAK_SECONDS", "10"))
    calls = failed = 0
    while time.time() < t_end:
        pl = rng.choice([16 << 10, 64 << 10, 256 << 10, 1 << 20, 2 << 20])
        d = tmp_path / f"s{calls}"
        d.mkdir()
        paths, sizes, exp = _torrent(str(d), rng, pl, 1000 + calls)
        n = len(exp) // 20
        want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
        first = rng.randint(0, n // 2)
        end = rng.randint(first, n)
        nctx = rng.choice([1, 1, 2, 3])
        threads = rng.choice([0, 1, 2, 4, 8])
        inject = rng.random() < 0.2
        pools = [HashPool(pl, slots=rng.choice([2, 3, 4]), slot_bytes=max(pl, rng.choice([4, 16, 64]) << 20),
                          hooks=inject) for _ in range(nctx)]
        try:
            if inject:
                pools[rng.randrange(nctx)].lib.vx_tuning_fail_launch_after(
                    pools[rng.randrange(nctx)]._h, rng.randint(0, 4))
            sp = Split(first, end, threads, rng.choice([0.0, 3e8, 2e9, 2e10]))
            out = {}

            def engines():
                try:
                    out["bad"] = (verify_files_split_multi(pools, paths, sizes, pl, exp, sp, io_threads=2 * nctx)
                                  if nctx > 1 else pools[0].verify_files_split(paths, sizes, pl, exp, sp,
                                                                               io_threads=rng.choice([1, 2, 4])))
                except VxError as e:
                    out["err"] = e

            th = threading.Thread(target=engines)
            th.start()
            if threads:
                oracle.pool_verify_files_claim(paths, sizes, pl, exp, threads, sp.claim_fn, sp.done_fn, sp.arg,
                                               first, sp.matched)
            th.join()
            got = sp.verdicts()
            if "err" in out:  # the caller verifies the engines' side itself
                failed += 1
                b = sp.boundary
                got[b - first:] = want[b:end]
            assert got == want[first:end], (pl, n, first, end, nctx, threads, sp.boundary)
            if not threads:
                assert sp.boundary == first or "err" in out
        finally:
            for p in pools:
                p.close()
        calls += 1
    assert calls >= 5
