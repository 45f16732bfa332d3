"""GPU: BASELINE config 5 end to end in the GPU suite, not only in bench.py.

The linux-mint.torrent geometry at full size (2,907,832,320 B, 1,387 x 2 MiB
pieces, last piece 1,179,648 B; synthetic bytes — the ISO is not available
offline) is written to a disk-backed directory and re-verified from disk by
``vx_verify_files`` — the engine's replacement for torrent.rs:724-740's
par_iter over check_piece_hash_sync (file_store.rs:228-303) — page-cache
warm and evicted (fsync + POSIX_FADV_DONTNEED: the reads go to the disk,
O_DIRECT where the filesystem takes it).  Every verdict is checked against
the CPU restatement of vortex's pool on the same file
(oracle.pool_verify_files), with:

* one damaged piece on disk (a flipped byte mid-file);
* the same bytes as a three-file torrent whose file boundaries fall inside
  pieces (file_store.rs's cross-file segments);
* that torrent's last file truncated, so the last piece cannot be read at
  all and the one before it is short: the reference's ``Err(_) => false``
  branch (torrent.rs:731-737), counted as I/O errors, not as mismatches;
* the self-balancing split (vx_verify_files_split) on the ISO, warm and cold,
  the pool stand-in claiming from the head beside the engine.
"""
import os

import pytest

import oracle

pytestmark = pytest.mark.gpu

PL = 2097152
TOTAL = 2907832320
DAMAGED = 700


def _copy_range(src: str, dst: str, off: int, length: int) -> None:
    with open(src, "rb") as fi, open(dst, "wb") as fo:
        fi.seek(off)
        left = length
        while left:
            b = fi.read(min(left, 64 << 20))
            assert b
            fo.write(b)
            left -= len(b)
        fo.flush()
        os.fsync(fo.fileno())


@pytest.mark.timeout(600)
def test_config5_full_size_from_disk(built, gpu):
    import bench
    from vortex_amd.hash_pool import HashPool

    threads = min(16, bench.cpu_share())
    d = bench.reverify_dir()
    iso = os.path.join(d, f"vx_cfg5_{os.getpid()}.iso")
    parts = [iso, iso + ".b", iso + ".c"]
    try:
        total, n, last = bench.write_linuxmint_file(iso)
        assert (total, n, last) == (TOTAL, 1387, 1179648)
        exp = oracle.pool_digest_synth(0x5EED0005, 0, n, PL, last_index=n - 1, last_len=last, threads=threads)
        with open(iso, "r+b") as f:  # one damaged piece
            f.seek(DAMAGED * PL + 4321)
            b = f.read(1)
            f.seek(DAMAGED * PL + 4321)
            f.write(bytes([b[0] ^ 0x20]))
            f.flush()
            os.fsync(f.fileno())

        with HashPool(PL, slots=4, slot_bytes=512 << 20, batch_pieces=4096) as pool:
            def check(paths, lens, want_bad_io, cold):
                if cold:
                    for p in paths:
                        bench.drop_cache(p)
                got, bad = pool.verify_files(paths, lens, PL, exp, io_threads=threads)
                if cold:
                    for p in paths:
                        bench.drop_cache(p)
                want = oracle.pool_verify_files(paths, lens, PL, exp, threads=threads)
                assert len(got) == n and got == want
                assert bad == want_bad_io
                return got

            # the ISO (one file), warm then cold
            for cold in (False, True):
                got = check([iso], [total], 0, cold)
                assert [i for i in range(n) if not got[i]] == [DAMAGED]

            # the split (vx_verify_files_split): the engine and the pool stand-in
            # at once, no plan, warm and cold; every verdict against the pool's
            for cold in (False, True):
                if cold:
                    bench.drop_cache(iso)
                call = bench.balanced_call(pool, [iso], [total], n, PL, exp, max(2, threads // 2),
                                           max(1, threads * 3 // 4), 2.0e9)
                assert call["matched"] == oracle.pool_verify_files([iso], [total], PL, exp, threads=threads)
                assert 0 <= call["boundary"] <= n and call["pool_pieces"] == call["boundary"]

            # the same bytes as three files whose boundaries fall inside pieces
            a = 1000 * PL + 12345
            b_len = 300 * PL - 777
            c_len = total - a - b_len
            _copy_range(iso, parts[1], a, b_len)
            _copy_range(iso, parts[2], a + b_len, c_len)
            os.truncate(iso, a)
            lens = [a, b_len, c_len]
            for cold in (False, True):
                got = check(parts, lens, 0, cold)
                assert [i for i in range(n) if not got[i]] == [DAMAGED]

            # the last file truncated: piece n-1 unreadable, piece n-2 short
            os.truncate(parts[2], c_len - last - 4096)
            for cold in (False, True):
                got = check(parts, lens, 2, cold)
                assert [i for i in range(n) if not got[i]] == [DAMAGED, n - 2, n - 1]
            st = pool.stats()
            assert st["io_errors"] == 4 and st["pieces_mismatched"] >= 6
    finally:
        for p in parts:
            if os.path.exists(p):
                os.unlink(p)
