"""The zero-copy slot path (vx_config.zero_copy = 1, the
default; slots of fewer than 128 pieces take the three-wave form, larger ones
the pair): a slot whose
pieces are all registered and 16-byte aligned is hashed straight out of host
memory by sha1_zc_split_kernel (cooperative 16-lane loads, LDS transpose),
with no gather kernel.  Every digest and verdict must equal hashlib's / the
oracle's on the download path (peer_connection.rs:1145-1158), with explicit
digests and with the device piece table, on ragged lengths that hit every
tail and padding case and a slot mixing short and long pieces; a slot with
one unregistered or unaligned piece must take the gather path instead and
still be exact."""
import hashlib
import mmap
import random

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

EDGE = [0, 1, 15, 16, 17, 55, 56, 63, 64, 65, 119, 120, 127, 128, 129, 255, 256, 257, 1023, 1024, 1025,
        4095, 4096, 65535, 65536, 65537, 200000, 262144, 262144 + 55, (1 << 20) + 3, 300]


def _pool_pieces(lens, seed, align_every=0):
    """Pieces at random 16-byte-aligned starts of a registered-to-be mmap,
    every `align_every`-th one shifted by 5 bytes (unaligned)."""
    rng = random.Random(seed)
    slot = max(lens) + 4096
    slot = (slot + 4095) // 4096 * 4096
    buf = mmap.mmap(-1, slot * (len(lens) + 4))
    np.frombuffer(buf, dtype=np.uint8)[:] = np.random.default_rng(seed).integers(0, 256, len(buf), dtype=np.uint8)
    order = list(range(len(lens) + 4))
    rng.shuffle(order)
    mv = memoryview(buf)
    pieces = []
    for k, L in enumerate(lens):
        start = order[k] * slot + 16 * rng.randrange(0, 64)
        if align_every and k % align_every == align_every - 1:
            start += 5
        pieces.append(mv[start:start + L])
    return buf, pieces


def _run_async(pool, pieces, want, bad_every=9, flush_every=10, table=False):
    for i, p in enumerate(pieces):
        exp = None if table else (want[i] if i % bad_every else bytes(20))
        pool.spawn(i, 7, p, len(p), exp)
        if i % flush_every == flush_every - 1:
            pool.flush()
    pool.drain()
    return {r.index: (r.hash_matched, r.digest) for r in pool.try_iter()}


# (batch_pieces, flush_every): 40-piece slots flushed every 10 pieces take the
# three-wave form; one 160-piece slot launched by the drain takes the pair
@pytest.mark.parametrize("form,batch,flush_every", [("loader", 40, 10), ("pair", 160, 1000)])
def test_zero_copy_async_ragged_exact(built, gpu, form, batch, flush_every):
    from vortex_amd import _lib
    from vortex_amd.hash_pool import HashPool

    lens = EDGE * 5
    random.Random(3).shuffle(lens)
    buf, pieces = _pool_pieces(lens, 11)
    want = [hashlib.sha1(p).digest() for p in pieces]
    assert want[5] == oracle.sha1(bytes(pieces[5]))
    with HashPool(2 << 20, slots=3, batch_pieces=batch, slot_bytes=16 << 20) as pool:
        pool.register_buffer(buf)
        z0 = pool.stats()["zero_copy_slots"]
        t0 = pool.stats()["gather_tiles"]
        got = _run_async(pool, pieces, want, flush_every=flush_every)
        zc = pool.stats()["zero_copy_slots"] - z0
        zl = pool.stats()["zero_copy_loader_slots"]
        tiles = pool.stats()["gather_tiles"] - t0
        pool.unregister_buffer(buf)
    assert len(got) == len(pieces)
    for i in range(len(pieces)):
        assert got[i][1] == want[i], (i, len(pieces[i]))
        assert got[i][0] == (i % 9 != 0), i
    assert zc >= len(pieces) // batch and tiles == 0  # every slot zero-copy, no gather
    assert (zl == zc) if form == "loader" else (zl < zc)


@pytest.mark.parametrize("batch", [64, 256])  # the three-wave form / the pair
def test_zero_copy_piece_table_and_batch(built, gpu, batch):
    """The device piece table (vx_submit_piece) on zero-copy slots, and a
    synchronous batch of short pieces (the slot path of vx_sha1_batch, which
    goes zero-copy too: vx_hash.h)."""
    from vortex_amd import _lib
    from vortex_amd.hash_pool import HashPool

    lens = [65536] * 200 + [1000, 64, 0, 65536 - 7]
    buf, pieces = _pool_pieces(lens, 12)
    want = [hashlib.sha1(p).digest() for p in pieces]
    table = bytearray(b"".join(want))
    for i in range(0, len(lens), 13):  # these must mismatch
        table[20 * i] ^= 1
    with HashPool(1 << 16, slots=4, batch_pieces=batch) as pool:
        pool.register_buffer(buf)
        pool.set_piece_table(bytes(table))
        z0 = pool.stats()["zero_copy_slots"]
        got = _run_async(pool, pieces, want, table=True, flush_every=17 if batch == 64 else 1000)
        z1 = pool.stats()["zero_copy_slots"]
        dig = pool.sha1_batch(pieces)
        zc = pool.stats()["zero_copy_slots"] - z0
        pool.unregister_buffer(buf)
    for i in range(len(pieces)):
        assert got[i] == (i % 13 != 0, want[i]), i
    assert dig == want
    assert z1 > z0 and zc > z1 - z0  # the async slots and the host batch's slots


def test_zero_copy_mixed_slots_fall_back(built, gpu):
    """Unaligned registered pieces and unregistered ones keep a slot off the
    zero-copy kernel (gather / DMA / stage as before); results stay exact."""
    from vortex_amd import _lib
    from vortex_amd.hash_pool import HashPool

    lens = EDGE * 3
    random.Random(4).shuffle(lens)
    buf, pieces = _pool_pieces(lens, 13, align_every=7)
    extra = [bytearray(oracle.gen_piece(13, k, L)) for k, L in enumerate([70000, 16, 0, 65536])]
    allp = pieces + extra
    want = [hashlib.sha1(p).digest() for p in allp]
    with HashPool(2 << 20, slots=3, batch_pieces=24, slot_bytes=16 << 20) as pool:
        pool.register_buffer(buf)
        t0 = pool.stats()["gather_tiles"]
        got = _run_async(pool, allp, want)
        tiles = pool.stats()["gather_tiles"] - t0
        pool.unregister_buffer(buf)
    for i in range(len(allp)):
        assert got[i] == (i % 9 != 0, want[i]), i
    assert tiles > 0


def test_zero_copy_config1_shape(built, gpu):
    """Config 1's shape on the zero-copy path: 1,024 x 256 KiB synthetic
    pieces in separately registered mmaps, shuffled, 1 % corrupted, against
    the oracle's pool."""
    from vortex_amd import _lib
    from vortex_amd.hash_pool import HashPool

    n, plen, seed, every = 1024, 256 * 1024, 0x5EED0001, 100
    bufs = []
    for i in range(n):
        m = mmap.mmap(-1, plen)
        m[:] = oracle.gen_piece(seed, i, plen, corrupt_every=every)
        bufs.append(m)
    clean = oracle.pool_digest_synth(seed, 0, n, plen, threads=8)
    order = list(range(n))
    random.Random(5).shuffle(order)
    with HashPool(plen) as pool:
        for m in bufs:
            pool.register_buffer(m)
        z0 = pool.stats()["zero_copy_slots"]
        for k, i in enumerate(order):
            pool.spawn(i, 1, bufs[i], plen, clean[20 * i:20 * i + 20])
            if k % 64 == 63:
                pool.flush()
        pool.drain()
        got = {r.index: (r.hash_matched, r.digest) for r in pool.try_iter()}
        zc = pool.stats()["zero_copy_slots"] - z0
        for m in bufs:
            pool.unregister_buffer(m)
    want = oracle.pool_digest_synth(seed, 0, n, plen, corrupt_every=every, threads=8)
    assert len(got) == n and zc > 0
    for i in range(n):
        assert got[i][1] == want[20 * i:20 * i + 20], i
        assert got[i][0] == (0 if oracle.is_corrupt(i, every) else 1), i


@pytest.mark.parametrize("plen,batch,zero_copy", [(16384, 128, 1), (262144, 128, 1), (2 << 20, 128, 1),
                                                  (16384, 32, 1), (262144, 32, 1), (262144, 128, 0), (16384, 32, 0)])
def test_zero_copy_default_policy(built, gpu, plen, batch, zero_copy):
    """With zero_copy = 1 (vx_config_default) a slot of registered aligned
    pieces goes zero-copy at every length and batch size (vx_engine.hip
    launch_slot_impl; small batches in the three-wave form) and never touches
    the gather; with zero_copy = 0 the same pieces are gathered into HBM
    first.  Every digest and verdict is hashlib's either way."""
    from vortex_amd import _lib
    from vortex_amd.hash_pool import HashPool

    n = 256
    expect_zc = zero_copy == 1
    buf, pieces = _pool_pieces([plen] * n, 21)
    want = [hashlib.sha1(p).digest() for p in pieces]
    with HashPool(plen, slots=3, batch_pieces=batch, slot_bytes=max(128 << 20, batch * plen),
                  zero_copy=zero_copy) as pool:
        pool.register_buffer(buf)
        got = _run_async(pool, pieces, want, flush_every=batch)
        zc = pool.stats()["zero_copy_slots"]
        st = pool.stats()
        pool.unregister_buffer(buf)
    for i in range(n):
        assert got[i] == (i % 9 != 0, want[i]), i
    assert (zc > 0) == expect_zc and (st["gather_tiles"] == 0) == expect_zc and st["staged_bytes"] == 0
