"""GPU: host-batch error paths and the multi-threaded stage copy.

* A host batch that fails part way (here: an injected VX_ENOMEM at the k-th
  submit, the non-latching error a failed pinned-stage allocation gives)
  returns only after every slot that was reading the caller's buffers has
  finished, and leaves nothing pending: vx_poll returns nothing, buffers can
  be unregistered (no EBUSY) and the next batch is bit-exact.
* Unregistered pieces of a host batch are copied into the pinned stage at
  launch by up to 16 threads (stage_copies); slots of 64 MiB and more split
  the copy, and the result must still be bit-exact.
* register_buffer refuses read-only objects and unregisters by object.
* A device failure in mid-stream (injected launch failure) leaves a dead
  context that still returns every finished result, names exactly the pieces
  to re-hash, and is destroyed cleanly.
* One ownership rule for submits (vx_hash.h): a piece is taken iff the submit
  returns 0, so every piece comes back exactly once — polled, refused with
  its buffer, or unfinished after a device failure.
"""
import hashlib
import mmap
import random
import time

import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fail_at", [0, 1, 37, 150, 299])
def test_batch_failure_part_way_leaves_clean_context(built, gpu, fail_at):
    from vortex_amd._lib import VX_ENOMEM, VxError, lib
    from vortex_amd.hash_pool import HashPool

    rng = random.Random(fail_at)
    plen = 100_000
    n = 300
    lens = [rng.choice([plen, plen, 64, 0, 4097, 77_777]) for _ in range(n)]
    reg = mmap.mmap(-1, n * 100_352)  # registered pool: one region, pieces 16-byte aligned
    pieces, keep = [], []
    for i, L in enumerate(lens):
        body = oracle.gen_piece(0xE1, i, L)
        if i % 2:
            off = i * 100_352
            reg[off:off + L] = body
            pieces.append(memoryview(reg)[off:off + L])
        else:
            pieces.append(bytearray(body))
        keep.append(body)
    want = [hashlib.sha1(b).digest() for b in keep]
    # slot_bytes 1 MiB: ~10 pieces per slot, so several slots are in flight when the failure hits
    with HashPool(plen, slots=3, batch_pieces=8, slot_bytes=1 << 20, hooks=True) as pool:
        pool.register_buffer(reg)
        pool.lib.vx_tuning_fail_submit_after(pool._h, fail_at)
        with pytest.raises(VxError) as e:
            pool.verify_batch(pieces, want)
        assert e.value.code == VX_ENOMEM
        assert pool.pending == 0
        assert pool.try_iter() == []
        pool.lib.vx_tuning_fail_submit_after(pool._h, -1)
        matched, dig = pool.verify_batch(pieces, want)
        assert matched == [True] * n and dig == want
        pool.unregister_buffer(reg)  # nothing in flight: must not be EBUSY
    # the failure also hits the async path without latching the context
    with HashPool(plen, slots=2, batch_pieces=4, hooks=True) as pool:
        pool.lib.vx_tuning_fail_submit_after(pool._h, 3)
        bufs = [bytearray(keep[i]) for i in range(6)]
        for i in range(3):
            pool.spawn(i, 0, bufs[i], len(bufs[i]), want[i])
        with pytest.raises(VxError):
            pool.spawn(3, 0, bufs[3], len(bufs[3]), want[3])
        pool.spawn(3, 0, bufs[3], len(bufs[3]), want[3])
        pool.drain()
        got = {r.index: r.hash_matched for r in pool.try_iter()}
        assert got == {0: True, 1: True, 2: True, 3: True}


def test_stage_copy_threads_large_slots(built, gpu):
    """Unregistered host batch through 96 MiB slots: every launch splits its
    stage copy over several threads (>= 16 MiB per thread)."""
    from vortex_amd.hash_pool import HashPool

    rng = random.Random(7)
    lens = [rng.choice([1 << 20, (1 << 20) - 13, 262_144, 16_384, 999]) for _ in range(400)]
    pieces = [oracle.gen_piece(0x57A6, i, L) for i, L in enumerate(lens)]
    bufs = [bytearray(p) for p in pieces]
    want = [hashlib.sha1(p).digest() for p in pieces]
    exp = list(want)
    exp[123] = bytes(20)
    with HashPool(1 << 20, slots=3, slot_bytes=96 << 20) as pool:
        matched, dig = pool.verify_batch(bufs, exp)
        assert dig == want
        assert matched == [i != 123 for i in range(len(pieces))]
        assert pool.sha1_batch(bufs) == want


def test_register_buffer_object_semantics(built, gpu):
    from vortex_amd.hash_pool import HashPool

    with HashPool(4096) as pool:
        with pytest.raises(ValueError):
            pool.register_buffer(b"\0" * 8192)  # read-only: would pin a private copy
        ba = bytearray(8192)
        pool.register_buffer(ba)
        with pytest.raises(ValueError):
            pool.register_buffer(ba)
        with pytest.raises(ValueError):
            pool.unregister_buffer(bytearray(8192))  # a different object
        body = oracle.gen_piece(1, 2, 4000)
        ba[:4000] = body
        pool.spawn(0, 0, memoryview(ba)[:4096], 4000, hashlib.sha1(body).digest())
        pool.drain()
        assert [r.hash_matched for r in pool.try_iter()] == [True]
        pool.unregister_buffer(ba)
        pool.register_buffer(ba)  # registrable again after unregistering
        pool.unregister_buffer(ba)


def test_ragged_layout_validation(built, gpu):
    """device.sha1_ragged refuses layouts the kernels would read out of
    bounds with (the raw C entries do not validate device metadata,
    vx_hash.h), and hashes a valid layout bit-exactly."""
    import torch

    from vortex_amd import device as vdev

    body = oracle.gen_piece(0xA1, 0, 4096)
    data = torch.frombuffer(bytearray(body), dtype=torch.uint8).to(gpu)

    def run(offs, lens, order=None, validate=True):
        o = torch.tensor(offs, dtype=torch.int64, device=gpu)
        ln = torch.tensor(lens, dtype=torch.int32, device=gpu)
        od = torch.tensor(order, dtype=torch.int32, device=gpu) if order is not None else None
        dig, _ = vdev.sha1_ragged(data, o, ln, order=od, validate=validate)
        torch.cuda.synchronize()
        return dig.cpu().numpy().tobytes()

    offs, lens = [0, 16, 4000, 4096], [10, 4080, 96, 0]
    want = b"".join(hashlib.sha1(body[o:o + L]).digest() for o, L in zip(offs, lens))
    assert run(offs, lens) == want
    assert run(offs, lens, order=[1, 2, 0, 3]) == want
    assert run(offs, lens, validate=False) == want
    for bad in ([0, 8], [0, -16]):  # misaligned, negative
        with pytest.raises(ValueError):
            run(bad, [1, 1])
    with pytest.raises(ValueError):
        run([0, 4080], [10, 17])  # ends at 4097 > 4096
    with pytest.raises(ValueError):
        run([0, 16], [1, -1])
    with pytest.raises(ValueError):
        run([0, 16], [1, 1], order=[0, 2])
    with pytest.raises(ValueError):
        run([0, 16], [1, 1], order=[0])
    with pytest.raises(ValueError):
        vdev.sha1_uniform(data, 2, 2049, stride=2064)  # 2064 + 2049 > 4096


def test_device_failure_recovery(built, gpu):
    """A device failure in mid-stream (injected: the 3rd launch fails as a
    device error would, vx_tuning_fail_launch_after) turns the context
    sticky.  The caller's recovery (INTEGRATION.md "Device failure"): every
    result the device did produce still comes back from vx_poll, then the
    error; the pieces whose result never came are exactly the ones to hash on
    vortex's own pool; destroying the context waits for the device to stop
    reading registered buffers, and a new context on the same GPU works."""
    import time

    from vortex_amd._lib import VX_EDEVICE, VxError, lib
    from vortex_amd.hash_pool import HashPool

    plen, n = 65536 + 32, 48
    pinned = mmap.mmap(-1, n * plen)
    bodies = [oracle.gen_piece(0xDEAD, i, plen) for i in range(n)]
    for i, b in enumerate(bodies):
        pinned[i * plen:(i + 1) * plen] = b
    digests = [hashlib.sha1(b).digest() for b in bodies]
    pool = HashPool(plen, slots=3, batch_pieces=8, hooks=True)
    pool.register_buffer(pinned)
    pool.lib.vx_tuning_fail_launch_after(pool._h, 2)
    results, refused = {}, None
    for i in range(n):
        try:
            pool.spawn(i, i, memoryview(pinned)[i * plen:(i + 1) * plen], plen, digests[i])
        except VxError as e:
            assert e.code == VX_EDEVICE
            refused = e.refused  # not taken: the piece comes back with the error (vx_hash.h ownership rule)
            break
    assert refused is not None and refused[0] == 23  # the third batch fills at the 24th submit and fails to launch
    time.sleep(0.5)  # the two launched batches finish
    for r in pool.try_iter():
        assert r.hash_matched and r.digest == digests[r.index]
        results[r.index] = True
    with pytest.raises(VxError) as ei:
        pool.try_iter()
    assert ei.value.code == VX_EDEVICE
    assert sorted(results) == list(range(16))
    assert pool.pending == 7  # a dead context's pending count = the pieces never returned
    lost = pool.take_unfinished()
    assert sorted(idx for idx, _, _ in lost) == list(range(16, 23))  # the refused piece is not among them
    for idx, _, buf in lost + [refused]:
        assert hashlib.sha1(bytes(buf[:plen])).digest() == digests[idx]  # the caller's pool takes over
    pool.close()  # waits for the streams, then unregisters and frees
    with HashPool(plen, slots=2, batch_pieces=8) as fresh:
        for i in range(10):
            fresh.spawn(i, i, bytearray(bodies[i]), plen, digests[i])
        fresh.drain()
        assert sorted(r.index for r in fresh.try_iter() if r.hash_matched) == list(range(10))


@pytest.mark.parametrize("mode", ["submit_enomem", "launch_in_submit", "launch_in_flush", "launch_two_slots"])
def test_submit_ownership_every_tag_once(built, gpu, mode):
    """vx_hash.h's ownership rule on the async path: a submit takes its piece
    iff it returns 0.  Whatever fails — a non-sticky VX_ENOMEM at a submit
    (vx_tuning_fail_submit_after), a launch failing inside vx_submit (the
    batch-full launch), inside vx_flush, or the lazy launch inside vx_poll
    (vx_tuning_fail_launch_after) — every piece comes back exactly once: as a
    completion from vx_poll, as the refused piece of a failed spawn, or from
    take_unfinished() after the context died.  Nothing is added by hand; at the
    end vx_pending() is 0 (usable context) or the unfinished count (dead one)."""
    from vortex_amd._lib import VX_EDEVICE, VX_ENOMEM, VxError, lib
    from vortex_amd.hash_pool import HashPool

    plen, n = 65536 + 48, 96
    reg = mmap.mmap(-1, n * plen)  # odd pieces come from a registered (gathered) region, even ones are staged
    bodies = [oracle.gen_piece(0x0E5, i, plen) for i in range(n)]
    bufs = []
    for i, b in enumerate(bodies):
        if i % 2:
            reg[i * plen:(i + 1) * plen] = b
            bufs.append(memoryview(reg)[i * plen:(i + 1) * plen])
        else:
            bufs.append(bytearray(b))
    digests = [hashlib.sha1(b).digest() for b in bodies]
    exp = [d if i % 13 else bytes(20) for i, d in enumerate(digests)]  # some planted mismatches
    # slots=2: vx_flush defers its launch while the other slot is in flight, so the
    # failing launch may be vx_poll's lazy one as well as vx_flush's or vx_submit's
    pool = HashPool(plen, slots=2 if mode == "launch_two_slots" else 3, batch_pieces=8, hooks=True)
    pool.register_buffer(reg)
    if mode == "submit_enomem":
        fails = {5, 6, 30, 71}  # non-sticky: the context stays usable after each
    elif mode == "launch_in_submit":
        pool.lib.vx_tuning_fail_launch_after(pool._h, 2)
    else:
        pool.lib.vx_tuning_fail_launch_after(pool._h, 3)
    seen: dict[int, str] = {}
    dead = False

    def take(results):
        for r in results:
            assert r.index not in seen, f"piece {r.index} returned twice"
            seen[r.index] = "polled"
            assert r.digest == digests[r.index]
            assert r.hash_matched == (exp[r.index] == digests[r.index])

    for i in range(n):
        if mode == "submit_enomem" and i in fails:
            pool.lib.vx_tuning_fail_submit_after(pool._h, 0)
        try:
            pool.spawn(i, 7, bufs[i], plen, exp[i])
        except VxError as e:
            assert e.refused is not None and e.refused[0] == i and e.refused[2] is bufs[i]
            assert i not in seen
            seen[i] = "refused"
            if e.code == VX_EDEVICE:
                dead = True
                break
            assert mode == "submit_enomem" and e.code == VX_ENOMEM and i in fails
            continue
        if mode != "launch_in_submit" and i % 5 == 4:  # the event loop's turn: flush, then drain
            try:
                pool.flush()
                take(pool.try_iter())
            except VxError as e:
                assert e.code == VX_EDEVICE
                dead = True
                break
    if not dead:
        assert mode == "submit_enomem"
        pool.drain()
        take(pool.try_iter())
        assert pool.pending == 0
    else:
        assert mode != "submit_enomem"
        time.sleep(0.3)  # batches launched before the failure finish
        while True:  # a dead context hands out every finished result, then the error
            try:
                got = pool.try_iter()
            except VxError as e:
                assert e.code == VX_EDEVICE
                break
            take(got)
        unfinished = pool.pending
        lost = pool.take_unfinished()
        assert len(lost) == unfinished
        for idx, conn, buf in lost:
            assert idx not in seen, f"piece {idx} both returned and unfinished"
            assert conn == 7 and buf is bufs[idx]
            seen[idx] = "unfinished"
    submitted = max(seen) + 1
    assert sorted(seen) == list(range(submitted)), "every submitted piece comes back exactly once"
    if mode == "submit_enomem":
        assert submitted == n and sorted(i for i, how in seen.items() if how == "refused") == sorted(fails)
    else:
        assert list(seen.values()).count("refused") <= 1 and "unfinished" in seen.values()
    pool.close()


def test_refuse_when_full_never_blocks(built, gpu):
    """vx_config.refuse_when_full = 1 (ABI 3): when every slot is in flight
    and the open batch is full, vx_submit returns VX_EBUSY at once instead of
    waiting for the oldest batch, so the event loop hands the piece to its
    own pool.  The documented invariant (vx_hash.h VX_EBUSY): the refused
    piece is not taken, vx_pending() is unchanged, and the only launch a
    refusal may make is the full open batch's (batches + 1, and then only
    when that batch held batch_pieces pieces).  Every piece is verified
    exactly once, on whichever side took it; the engine never stalls the
    submitting thread (submit_stall_ns == 0) and counts its refusals."""
    from vortex_amd._lib import VX_EBUSY, VxError
    from vortex_amd.hash_pool import HashPool

    plen, n = 1 << 20, 96
    bodies = [oracle.gen_piece(0xB5, i, plen) for i in range(n)]
    want = [hashlib.sha1(b).digest() for b in bodies]
    bufs = [bytearray(b) for b in bodies]
    for i in range(0, n, 7):  # some pieces corrupted after their expected digest was taken
        bufs[i][i % plen] ^= 0x40
    verdict_truth = [hashlib.sha1(bytes(b)).digest() == w for b, w in zip(bufs, want)]
    # 2 slots of 8 pieces: 16 pieces fill the pipeline, and 1 MiB chains keep it full for a while
    with HashPool(plen, slots=2, batch_pieces=8, slot_bytes=8 << 20, refuse_when_full=1) as pool:
        got, refused, launched_on_refusal = {}, [], 0
        taken = 0  # pieces the engine took; every launch before a refusal holds exactly 8
        for i in range(n):
            pend, batches = pool.pending, pool.stats()["batches"]
            try:
                pool.spawn(i, 7, bufs[i], plen, want[i])
                taken += 1
            except VxError as e:
                assert e.code == VX_EBUSY and e.refused[0] == i and e.refused[2] is bufs[i]
                refused.append(i)  # vortex's own pool hashes it (here: hashlib)
                got[i] = hashlib.sha1(bytes(bufs[i])).digest() == want[i]
                # the invariant: no piece changed owner; at most the full open batch launched
                assert pool.pending == pend
                delta = pool.stats()["batches"] - batches
                assert delta in (0, 1)
                if delta:
                    assert taken == 8 * (batches + 1), (taken, batches)  # the open batch was full
                    launched_on_refusal += 1
                else:
                    assert taken == 8 * batches  # nothing open was left unlaunched
        assert refused, "the pipeline never filled: no refusal to test"
        pool.drain()
        for r in pool.try_iter():
            assert r.index not in got and r.conn_id == 7
            got[r.index] = r.hash_matched
        assert sorted(got) == list(range(n))
        assert [got[i] for i in range(n)] == verdict_truth
        st = pool.stats()
        assert st["submits_refused"] == len(refused) and st["submit_stall_ns"] == 0
        assert st["pieces_completed"] == n - len(refused)
        # nothing in flight: a submit is taken again
        pool.spawn(0, 7, bytearray(bodies[0]), plen, want[0])
        pool.drain()
        (r,) = pool.try_iter()
        assert r.hash_matched


@pytest.mark.parametrize("copy_stream", [1, 0])
def test_chunk_round_failure_then_reuse_and_destroy(built, gpu, tmp_path, copy_stream):
    """A re-verify whose k-th chunk round fails after its data copy was
    queued (injected: vx_tuning_fail_launch_after, between the copy and the
    kernel launch), on the copy stream (verify_copy_stream = 1, the default)
    and on the slot streams (0).  The call returns the error only after the
    queued part of the round finished (a stale `done` event must
    not free a slot under a DMA); the same context's next call is bit-exact
    against the oracle on a file with a damaged piece; vx_destroy then waits
    for the copy stream before it frees the stages."""
    from vortex_amd._lib import VX_EDEVICE, VxError
    from vortex_amd.hash_pool import HashPool

    pl, n = 2 << 20, 24
    path = tmp_path / "t.bin"
    path.write_bytes(b"".join(oracle.gen_piece(0xC5, i, pl) for i in range(n)))
    exp = b"".join(oracle.sha1(oracle.gen_piece(0xC5, i, pl)) for i in range(n))
    with open(path, "r+b") as f:  # piece 9 damaged on disk
        f.seek(9 * pl + 12345)
        f.write(b"\x00\xff")
    want = oracle.pool_verify_files([str(path)], [n * pl], pl, exp, threads=4)
    assert sum(want) == n - 1
    for fail_at in (0, 5, 17):
        with HashPool(pl, slots=3, slot_bytes=8 << 20, verify_chunk=65536, hooks=True) as pool:
            pool.lib.vx_tuning_verify_copy_stream(pool._h, copy_stream)
            pool.lib.vx_tuning_fail_launch_after(pool._h, fail_at)
            with pytest.raises(VxError) as ei:
                pool.verify_files([str(path)], [n * pl], pl, exp, io_threads=4)
            assert ei.value.code == VX_EDEVICE and "injected" in str(ei.value)
            got, bad = pool.verify_files([str(path)], [n * pl], pl, exp, io_threads=4)
            assert got == want and bad == 0
            assert pool.stats()["chunk_rounds"] > fail_at
