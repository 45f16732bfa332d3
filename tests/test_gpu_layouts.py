"""GPU parity on the reference's own multi-file layouts.

Every layout of tests/golden/vectors.json `file_store_layouts` — the ten
FileStore tests of bittorrent/src/file_store.rs:567-760 (tiny piece lengths of
64 and 256 B, files shorter than a piece, files ending on piece boundaries,
a 16 B last piece), `disk_operations_for_all_valid_piece_indices`, the
integration geometries of bittorrent/tests/ (128 KiB and 16 KiB pieces) and
two extra edge layouts (zero-length files) — goes through the three GPU
paths that replace the reference's hashing:

* ``vx_verify_files``: the bulk re-verify from disk (torrent.rs:724-740 over
  file_store.rs:228-303), files in fixture order and reversed;
* ``vx_verify_batch``: host pieces (the par_iter verify over buffers);
* ``vx_submit``/``vx_poll``: the download path (peer_connection.rs:1145-1158).

Expected digests are hashlib over the concatenated files (the fixture pins
them for path order).  Bar: every verdict true, every digest bit-exact, and
one flipped byte fails exactly the piece that holds it.
"""
import hashlib

import pytest

from _layouts import flip_file_byte, flip_offset, materialize

pytestmark = pytest.mark.gpu


def _names():
    import json
    import os

    with open(os.path.join(os.path.dirname(__file__), "golden", "vectors.json")) as f:
        return [e["name"] for e in json.load(f)["file_store_layouts"]]


@pytest.mark.parametrize("name", _names())
def test_layout_all_gpu_paths(built, gpu, golden, tmp_path, name):
    from vortex_amd.hash_pool import HashPool

    e = next(x for x in golden["file_store_layouts"] if x["name"] == name)
    pl, n = e["piece_length"], e["num_pieces"]
    off = flip_offset(e)
    bad_piece = off // pl
    with HashPool(pl) as pool:
        for reverse in (False, True):
            root = tmp_path / ("rev" if reverse else "fwd")
            paths, lens, data, exp = materialize(e, root, reverse=reverse)
            # bulk re-verify from disk
            for io_threads in (1, 4):
                got, nbad = pool.verify_files(paths, lens, pl, exp, io_threads=io_threads)
                assert nbad == 0 and got == [True] * n, (name, reverse, io_threads)
            flip_file_byte(paths, lens, off)
            got, nbad = pool.verify_files(paths, lens, pl, exp)
            assert nbad == 0 and got == [i != bad_piece for i in range(n)], (name, reverse)
            # host batch over the pieces, one of them corrupted
            pieces = [bytearray(data[i:i + pl]) for i in range(0, len(data), pl)]
            want = [exp[20 * i:20 * i + 20] for i in range(n)]
            matched, dig = pool.verify_batch(pieces, want)
            assert matched == [True] * n and dig == want
            pieces[bad_piece][off - bad_piece * pl] ^= 0x5A
            matched, dig = pool.verify_batch(pieces, want)
            assert matched == [i != bad_piece for i in range(n)]
            assert dig[bad_piece] == hashlib.sha1(bytes(pieces[bad_piece])).digest()
            # download path: each piece in a piece_length-capacity buffer with
            # stale bytes past piece_len (buf_pool.rs:148-157)
            for i, p in enumerate(pieces):
                buf = bytearray(p) + b"\xEE" * (pl - len(p))
                pool.spawn(i, 7, buf, len(p), want[i])
            pool.drain()
            res = {r.index: (r.hash_matched, r.digest) for r in pool.try_iter()}
            assert sorted(res) == list(range(n))
            assert all(res[i][0] == (i != bad_piece) for i in range(n))
            assert all(res[i][1] == want[i] for i in range(n) if i != bad_piece)


def test_fresh_fallocated_files(built, gpu, tmp_path):
    """The re-verify vortex runs right after InitializedState::new, whose
    FileStore::new creates every file and fallocates it to its torrent
    length (file_store.rs:146, File::create at file_store.rs:22-43): regions
    not downloaded yet read as zeros.  A piece whose real content is all
    zeros therefore verifies true, pieces already written verify true, the
    rest false, and no piece is an I/O error — the reference's verdicts
    exactly (checked against the oracle's restatement too)."""
    import oracle
    from vortex_amd.hash_pool import HashPool

    pl = 64 * 1024
    sizes = [100_000, 3 * pl + 5, 17, 2 * pl]
    data = bytearray(oracle.gen_piece(0xFA11, 0, sum(sizes)))
    data[2 * pl:3 * pl] = bytes(pl)  # piece 2 really is all zeros
    n = (len(data) + pl - 1) // pl
    exp = b"".join(hashlib.sha1(bytes(data[i:i + pl])).digest() for i in range(0, len(data), pl))
    paths, acc = [], 0
    for k, L in enumerate(sizes):
        p = tmp_path / f"f{k}"
        with open(p, "wb") as f:
            f.truncate(L)  # what fallocate leaves: L zero bytes
        paths.append(str(p))
    written = {0, 4}  # pieces the client already wrote (Write disk ops, file_store.rs:167-223)
    for i in written:
        lo, hi = i * pl, min((i + 1) * pl, len(data))
        acc = 0
        for p, L in zip(paths, sizes):
            a, b = max(lo, acc), min(hi, acc + L)
            if a < b:
                with open(p, "r+b") as f:
                    f.seek(a - acc)
                    f.write(bytes(data[a:b]))
            acc += L
    want = [i in written or i == 2 for i in range(n)]
    assert oracle.pool_verify_files(paths, sizes, pl, exp, threads=2) == want
    with HashPool(pl) as pool:
        got, nbad = pool.verify_files(paths, sizes, pl, exp)
    assert got == want and nbad == 0
