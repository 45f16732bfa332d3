"""GPU: BASELINE config 1's plumbing at its full size on the HIP path.

Config 1 is 4,096 x 256 KiB pieces through vortex's hashing-pool plumbing.
Here they go through the async download path exactly as vortex hands them
over: every piece in its own pool buffer (one AnonymousMmap per buffer,
buf_pool.rs:92-98, each registered with the engine), submitted in a shuffled
order as pieces complete (HashPool.spawn = scope.spawn, peer_connection.rs:
1145-1158), one flush + drain per event-loop turn (event_loop.rs:554-557 ->
torrent.rs:415-442).  1 % of the buffers carry one flipped byte.  Every
verdict and every digest is checked against the CPU oracle (the C
restatement of vortex's pool, oracle.pool_digest_synth) — 1 GiB, well under a
second of GPU time.
"""
import ctypes
import mmap
import random

import pytest

import oracle

pytestmark = pytest.mark.gpu

SEED, N, PLEN, CORRUPT = 0x5EED0001, 4096, 256 * 1024, 100


@pytest.mark.parametrize("table", [False, True])  # expected digest per spawn / device piece table
def test_config1_async_4096x256k(built, gpu, table):
    from vortex_amd.hash_pool import HashPool

    bufs = [mmap.mmap(-1, PLEN) for _ in range(N)]
    for i, b in enumerate(bufs):
        oracle.lib().vxo_gen_piece(SEED, i, PLEN, CORRUPT, ctypes.c_void_p(ctypes.addressof(ctypes.c_char.from_buffer(b))))
    clean = oracle.pool_digest_synth(SEED, 0, N, PLEN, threads=8)  # the torrent's `pieces` table
    actual = oracle.pool_digest_synth(SEED, 0, N, PLEN, corrupt_every=CORRUPT, threads=8)
    order = list(range(N))
    random.Random(1).shuffle(order)
    got = {}
    with HashPool(PLEN) as pool:
        from vortex_amd import _lib

        for b in bufs:
            pool.register_buffer(b)
        if table:
            pool.set_piece_table(clean)
        for k, i in enumerate(order):
            pool.spawn(i, i % 128, bufs[i], PLEN, None if table else clean[20 * i:20 * i + 20])
            if k % 64 == 63:  # one event-loop turn
                pool.flush()
                for r in pool.try_iter():
                    assert r.index not in got
                    got[r.index] = r
        pool.drain()
        for r in pool.try_iter():
            assert r.index not in got
            got[r.index] = r
        assert pool.pending == 0
        st = pool.stats()
        zc = pool.stats()["zero_copy_slots"]
        for b in bufs:
            pool.unregister_buffer(b)
    assert sorted(got) == list(range(N))
    bad = sorted(i for i, r in got.items() if not r.hash_matched)
    assert bad == [i for i in range(N) if oracle.is_corrupt(i, CORRUPT)] and len(bad) == N // CORRUPT
    for i, r in got.items():
        assert r.digest == actual[20 * i:20 * i + 20], i
        assert r.conn_id == i % 128 and r.buffer is bufs[i]  # the buffer comes back with its piece
    assert st["pieces_completed"] == N and st["pieces_mismatched"] == len(bad)
    # registered buffers: pulled by the gather kernel or hashed in place (zero-copy slots), never staged
    assert st["gather_tiles"] + zc > 0 and st["staged_bytes"] == 0
