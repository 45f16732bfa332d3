"""GPU: vx_get_stats / vx_reset_stats (include/vx_hash.h "observability").

vortex's `metrics` feature has no hashing series; the engine's
counters must add up exactly to what each path did, whichever path ran:
the async submit/poll path (gather kernel for registered 16-byte aligned
pieces, pinned staging for the rest), host batches (whole-piece slots and
the strided chunk path), and the file re-verify (whole-piece and chunked,
with I/O errors).  Every count is checked against the test's own bookkeeping;
the latency histogram must account for every harvested batch.
"""
import hashlib
import mmap
import random
import sys

import pytest

import oracle
from conftest import ROOT

pytestmark = pytest.mark.gpu


def _check_latency(st):
    assert sum(st["batch_latency_hist"]) == st["batch_latency_count"]
    if st["batch_latency_count"]:
        assert st["batch_latency_max_us"] * st["batch_latency_count"] >= st["batch_latency_sum_us"]
        top = max(k for k, v in enumerate(st["batch_latency_hist"]) if v)
        assert st["batch_latency_max_us"] >> top in (1, 0) or top == len(st["batch_latency_hist"]) - 1


def test_stats_async_path(built, gpu):
    from vortex_amd.hash_pool import HashPool

    rng = random.Random(8)
    plen = 16384 * 3 + 96  # 16-byte multiple: registered pieces go through the gather kernel
    # zero_copy=0: counts the gather kernel's tiles (zero-copy slots: test_gpu_zero_copy.py)
    with HashPool(plen, slots=2, batch_pieces=7, zero_copy=0) as pool:
        st0 = pool.stats()
        assert all(v == 0 for k, v in st0.items() if k != "batch_latency_hist")
        pinned = mmap.mmap(-1, plen * 40)
        pool.register_buffer(pinned)
        total, staged, tiles, bad = 0, 0, 0, 0
        got = {}
        for i in range(120):
            L = plen if i % 11 else rng.randint(0, plen)
            body = oracle.gen_piece(0x57A7, i, L)
            if i < 40:
                view = memoryview(pinned)[i * plen:(i + 1) * plen]
                view[:L] = body
                buf = view
                tiles += 1 if L else 0
            else:
                buf = bytearray(body)
                staged += L
            exp = hashlib.sha1(body).digest() if i % 13 else bytes(20)
            bad += i % 13 == 0
            total += L
            pool.spawn(i, i, buf, L, exp)
            if i % 17 == 0:
                pool.flush()
                for r in pool.try_iter():
                    got[r.index] = r.hash_matched
        pool.drain()
        for r in pool.try_iter():
            got[r.index] = r.hash_matched
        assert len(got) == 120 and sum(not m for m in got.values()) == bad
        st = pool.stats()
        assert st["pieces_completed"] == 120
        assert st["pieces_mismatched"] == bad
        assert st["bytes_completed"] == total
        assert st["staged_bytes"] == staged
        assert st["gather_tiles"] == tiles
        assert st["batches"] >= 120 // 7 and st["batch_latency_count"] == st["batches"]
        assert st["chunk_rounds"] == 0 and st["io_errors"] == 0
        _check_latency(st)
        pool.unregister_buffer(pinned)
        pool.reset_stats()
        st = pool.stats()
        assert all(v == 0 for k, v in st.items() if k != "batch_latency_hist")
        assert not any(st["batch_latency_hist"])


def test_stats_submit_stall(built, gpu):
    """Two slots of 4 pieces: the 9th submit finds both in flight and blocks
    on the oldest batch — the event-loop stall the counter reports."""
    from vortex_amd.hash_pool import HashPool

    plen = 1 << 20
    body = bytearray(oracle.gen_piece(3, 0, plen))
    good = hashlib.sha1(body).digest()
    with HashPool(plen, slots=2, batch_pieces=4) as pool:
        for i in range(12):
            pool.spawn(i, 0, body, plen, good)
        pool.drain()
        assert len(pool.try_iter()) == 12
        st = pool.stats()
        assert st["submit_stall_ns"] > 0
        assert st["pieces_completed"] == 12 and st["pieces_mismatched"] == 0
        _check_latency(st)


def test_stats_host_batches(built, gpu):
    from vortex_amd.hash_pool import HashPool

    rng = random.Random(9)
    lens = [rng.choice([0, 64, 4097, 65536, 200_000]) for _ in range(150)]
    pieces = [oracle.gen_piece(0xB7, i, L) for i, L in enumerate(lens)]
    exp = [hashlib.sha1(p).digest() if i % 9 else b"\x01" * 20 for i, p in enumerate(pieces)]
    with HashPool(200_000, slots=3) as pool:
        matched, _ = pool.verify_batch([bytearray(p) for p in pieces], exp)
        assert [not m for m in matched] == [i % 9 == 0 for i in range(150)]
        st = pool.stats()
        assert st["pieces_completed"] == 150
        assert st["pieces_mismatched"] == sum(i % 9 == 0 for i in range(150))
        assert st["bytes_completed"] == sum(lens)
        assert st["staged_bytes"] == sum(lens)
        _check_latency(st)

    # long equal pieces at a constant stride in one registered mmap: the strided chunk path
    n, L = 24, (3 << 20) + 48
    region = mmap.mmap(-1, n * L)
    for i in range(n):
        region[i * L:(i + 1) * L] = oracle.gen_piece(0xB8, i, L)
    views = [memoryview(region)[i * L:(i + 1) * L] for i in range(n)]
    exp = [hashlib.sha1(v).digest() if i != 5 else bytes(20) for i, v in enumerate(views)]
    with HashPool(L, slots=3) as pool:
        pool.register_buffer(region)
        matched, _ = pool.verify_batch(views, exp)
        assert [not m for m in matched] == [i == 5 for i in range(n)]
        st = pool.stats()
        assert st["chunk_rounds"] > 0
        assert (st["pieces_completed"], st["pieces_mismatched"], st["bytes_completed"]) == (n, 1, n * L)
        pool.unregister_buffer(region)


@pytest.mark.parametrize("pl", [65536, 1 << 20])  # whole-piece slots / resumable chunk rounds
def test_stats_reverify(built, gpu, tmp_path, pl):
    from vortex_amd.hash_pool import HashPool

    lens = [5 * pl + 1000, 3 * pl - 7, 2 * pl]
    data = [oracle.gen_piece(0xF1, k, L) for k, L in enumerate(lens)]
    paths = []
    for k, d in enumerate(data):
        p = tmp_path / f"f{k}"
        p.write_bytes(d if k != 1 else d[:pl])  # file 1 is short: its missing bytes are I/O errors
        paths.append(str(p))
    whole = b"".join(data)
    n = (len(whole) + pl - 1) // pl
    exp = bytes(20) + b"".join(hashlib.sha1(whole[i * pl:(i + 1) * pl]).digest() for i in range(1, n))
    with HashPool(pl, slots=4) as pool:
        got, nbad = pool.verify_files(paths, lens, pl, exp)
        # piece 0 reads fine but its expected digest is wrong; the short file's pieces are I/O errors
        assert nbad > 0 and not got[0] and sum(not g for g in got) == nbad + 1
        st = pool.stats()
        assert st["pieces_completed"] == n
        assert st["bytes_completed"] == len(whole)
        assert st["io_errors"] == nbad
        assert st["pieces_mismatched"] == 1  # I/O errors are counted once, in io_errors
        assert (st["chunk_rounds"] > 0) == (pl >= 1 << 20)
        _check_latency(st)
        # the call's time budget (vx_last_verify, recorded per call by bench.py)
        tr = pool.last_verify()
        assert tr["read_bytes"] == len(whole)  # every piece byte requested once (failed reads included)
        assert 0 < tr["read_busy_ms"] and 0 < tr["first_read_ms"] <= tr["wall_ms"] and tr["read_span_ms"] <= tr["wall_ms"]
        assert 1 <= tr["readers"] <= 16
        if pl >= 1 << 20:  # chunk rounds: GPU-timed copies of the staged bytes
            assert tr["rounds"] == st["chunk_rounds"] and tr["copy_bytes"] >= len(whole)
            assert 0 < tr["copy_busy_ms"] <= tr["copy_span_ms"] + 1e-3 and 0 < tr["copy_busy_frac"] <= 1.0001
        else:
            assert tr["rounds"] == 0 and tr["copy_bytes"] == 0
        # the round timeline (vx_last_verify_rounds): one record per timed round, times on the
        # call's clock in order: reads queued <= done <= enqueued; copy start <= end <= kernel end
        rounds = pool.last_verify_rounds()
        if pl < 1 << 20:
            assert rounds == []
        else:
            from vortex_amd._lib import VX_ROUND_HEAD_RAMP, VX_ROUND_NEW_WINDOW, VX_ROUND_TAIL_RAMP

            assert len(rounds) == tr["rounds"] and sum(r["bytes"] for r in rounds) == tr["copy_bytes"]
            assert rounds[0]["flags"] & VX_ROUND_NEW_WINDOW and rounds[0]["offset"] == 0
            assert any(r["flags"] & VX_ROUND_HEAD_RAMP for r in rounds) and rounds[-1]["flags"] & VX_ROUND_TAIL_RAMP
            slack = 0.5  # ms: the GPU-to-host clock mapping's error (the anchor event's dispatch latency)
            for a, b in zip(rounds, rounds[1:]):
                assert b["copy_start_ms"] >= a["copy_end_ms"] - 1e-3  # copies are chained across slots
                assert b["enqueue_ms"] >= a["enqueue_ms"]
            for r in rounds:
                assert 0 <= r["read_submit_ms"] <= r["read_done_ms"] <= r["enqueue_ms"] <= tr["wall_ms"]
                assert r["enqueue_ms"] - slack <= r["copy_start_ms"] <= r["copy_end_ms"] <= r["kernel_end_ms"]
                assert r["kernel_end_ms"] <= tr["wall_ms"] + slack and r["lanes"] >= 1
            sys.path.insert(0, ROOT)
            import bench

            gaps = bench.copy_gaps(rounds)
            assert gaps["rounds"] == len(rounds) and gaps["gap_ms"] >= 0
            assert set(gaps["by_cause"]) <= {"read", "hand-off", "device"}
