"""CPU: pin the oracle (oracle/) against the golden vectors before trusting it.

Golden sources (tests/golden/make_golden.py): FIPS 180-4 vectors, hashlib
digests of boundary lengths, the reference's implicit known answers
(bittorrent/src/lib.rs setup_test / setup_seeding_test), the
pure-Python synthetic-piece spec and the linux-mint.torrent geometry.
"""
import hashlib
import os

import pytest

import oracle

BACKENDS = [1, 2] if oracle.has_shani() else [1]


def pattern(n):
    return bytes(((i * 131 + 7) & 0xFF) for i in range(n))


@pytest.mark.parametrize("backend", BACKENDS)
def test_fips_vectors(golden, backend):
    for v in golden["fips"]:
        assert oracle.sha1_backend(bytes.fromhex(v["hex_input"]), backend).hex() == v["sha1"], v["name"]
    m = golden["million_a"]
    assert oracle.sha1_backend(bytes([m["byte"]]) * m["len"], backend).hex() == m["sha1"]


@pytest.mark.parametrize("backend", BACKENDS)
def test_boundary_lengths(golden, backend):
    for v in golden["boundary"]:
        assert oracle.sha1_backend(pattern(v["len"]), backend).hex() == v["sha1"], v["len"]


def test_streaming_equals_oneshot(golden):
    data = pattern(70000)
    for chunk in (1, 63, 64, 65, 777, 16384):
        h = oracle.Sha1Stream()
        for i in range(0, len(data), chunk):
            h.update(data[i:i + chunk])
        assert h.finalize() == hashlib.sha1(data).digest(), chunk


def test_reference_setup_test(golden):
    st = golden["setup_test"]
    data = bytes([st["files"][0]["byte"]]) * st["files"][0]["len"]
    pl = st["piece_length"]
    got = [oracle.sha1(data[i:i + pl]).hex() for i in range(0, len(data), pl)]
    assert got == st["pieces"]
    assert got[0] == "0b5f75802398863cb57d24b30c5caa55e56062b6"


def test_reference_seeding_layout(golden, tmp_path):
    """setup_seeding_test: 3 files, piece 0 spans all three, last piece 164 B.
    Checked through the file_store.rs:228-303 restatement (pread + stream)."""
    st = golden["setup_seeding_test"]
    paths, lens = [], []
    for k, f in enumerate(st["files"]):
        p = tmp_path / f"f{k + 1}.txt"
        p.write_bytes(bytes([f["byte"]]) * f["len"])
        paths.append(str(p))
        lens.append(f["len"])
    pl = st["piece_length"]
    total = sum(lens)
    n = (total + pl - 1) // pl
    assert n == len(st["pieces"]) == 9
    assert oracle.piece_len(8, n, pl, total) == 164
    assert oracle.piece_segments(0, lens, pl) == [(0, 0, 64), (1, 0, 100), (2, 0, pl - 164)]
    for i in range(n):
        assert oracle.check_piece_hash_sync(paths, lens, pl, i, bytes.fromhex(st["pieces"][i])), i
    # a wrong expected digest is a `false` verdict, not an error
    assert not oracle.check_piece_hash_sync(paths, lens, pl, 3, b"\0" * 20)


def test_piece_len_rule(golden):
    lm = golden["linux_mint"]
    n, pl, total = lm["num_pieces"], lm["piece_length"], lm["length"]
    assert oracle.piece_len(0, n, pl, total) == pl
    assert oracle.piece_len(n - 1, n, pl, total) == lm["last_piece_len"] == 1179648
    # exact multiple: last piece is a full piece (piece_selector.rs:66-69)
    assert oracle.piece_len(3, 4, 100, 400) == 100


def test_linux_mint_table_fixture(golden):
    lm = golden["linux_mint"]
    path = os.path.join(os.path.dirname(__file__), "golden", "linux_mint_pieces.bin")
    table = open(path, "rb").read()
    assert len(table) == 20 * lm["num_pieces"]
    assert hashlib.sha1(table).hexdigest() == lm["pieces_sha1_of_table"]
    assert table[:20].hex() == lm["first_pieces"][0]


def test_synthetic_generator_spec(golden):
    for v in golden["synthetic"]:
        data = oracle.gen_piece(v["seed"], v["piece"], v["len"], v["corrupt_every"])
        assert data[:32].hex() == v["head_hex"][: 2 * min(32, v["len"])]
        assert hashlib.sha1(data).hexdigest() == v["sha1"], v


def test_pool_restatement_matches_hashlib():
    pieces = [pattern(n) for n in (0, 1, 55, 56, 64, 1000, 32768, 100000)]
    exp = b"".join(hashlib.sha1(p).digest() for p in pieces)
    bad = bytearray(exp)
    bad[20 * 3] ^= 1
    dig, matched = oracle.pool_verify(pieces, bytes(bad), threads=3)
    assert dig == exp
    assert matched == [True, True, True, False, True, True, True, True]


def test_pool_digest_synth_matches_generator():
    n, plen = 33, 5000
    got = oracle.pool_digest_synth(0x5EED0002, 100, n, plen, last_index=132, last_len=77, corrupt_every=10,
                                   threads=4)
    for i in range(n):
        g = 100 + i
        L = 77 if g == 132 else plen
        assert got[20 * i:20 * i + 20] == hashlib.sha1(oracle.gen_piece(0x5EED0002, g, L, 10)).digest()


def _write_files(tmp_path, sizes, seed=3):
    paths = []
    for k, L in enumerate(sizes):
        p = tmp_path / f"file{k}.bin"
        p.write_bytes(oracle.gen_piece(seed, k, L))
        paths.append(str(p))
    return paths


def _expected_from_concat(paths, sizes, pl):
    data = b"".join(open(p, "rb").read() for p in paths)
    assert len(data) == sum(sizes)
    return b"".join(hashlib.sha1(data[i:i + pl]).digest() for i in range(0, len(data), pl))


def test_pool_verify_files_restatement(tmp_path):
    """The C++ bulk re-verify restatement agrees with the per-piece Python
    restatement of check_piece_hash_sync, including missing/short files."""
    sizes = [64, 100, 0, 5000, 32768, 3, 40000]
    pl = 4096
    paths = _write_files(tmp_path, sizes)
    exp = _expected_from_concat(paths, sizes, pl)
    n = len(exp) // 20
    got = oracle.pool_verify_files(paths, sizes, pl, exp, threads=3)
    assert got == [True] * n
    want = [oracle.check_piece_hash_sync(paths, sizes, pl, i, exp[20 * i:20 * i + 20]) for i in range(n)]
    assert want == got
    # truncate file 4 and delete file 6: pieces touching them turn false
    with open(paths[4], "r+b") as f:
        f.truncate(30000)
    os.unlink(paths[6])
    got = oracle.pool_verify_files(paths, sizes, pl, exp, threads=3)
    spans = {i: {fi for fi, _, _ in oracle.piece_segments(i, sizes, pl)} for i in range(n)}
    for i in range(n):
        touches_bad = 6 in spans[i] or any(fi == 4 and off + ln > 30000 for fi, off, ln in
                                          oracle.piece_segments(i, sizes, pl))
        assert got[i] == (not touches_bad), i


def _layout_ids(golden_path=os.path.join(os.path.dirname(__file__), "golden", "vectors.json")):
    import json

    with open(golden_path) as f:
        return [e["name"] for e in json.load(f)["file_store_layouts"]]


@pytest.mark.parametrize("name", _layout_ids())
@pytest.mark.parametrize("reverse", [False, True])
def test_reference_file_store_layouts(golden, tmp_path, name, reverse):
    """The reference's own FileStore layouts (file_store.rs:567-760, the
    integration-test geometries) through the oracle's restatement of the
    walk (piece_segments, file_store.rs:240-298) and the C++ bulk re-verify
    pool (torrent.rs:724-740): segments equal the geometric interval
    intersection, every piece verifies, and one flipped byte fails exactly
    the piece that holds it."""
    from _layouts import flip_file_byte, flip_offset, interval_segments, materialize

    e = next(x for x in golden["file_store_layouts"] if x["name"] == name)
    paths, lens, data, exp = materialize(e, tmp_path, reverse=reverse)
    pl, n = e["piece_length"], e["num_pieces"]
    assert len(exp) == 20 * n and sum(lens) == e["total"]
    assert oracle.piece_len(n - 1, n, pl, e["total"]) == e["last_piece_len"]
    geo = e["segments"] if ("segments" in e and not reverse) else interval_segments(lens, pl)
    for i in range(n) if n <= 64 else (0, 1, n // 2, n - 2, n - 1):
        assert [list(s) for s in oracle.piece_segments(i, lens, pl)] == geo[i], i
    assert oracle.pool_verify_files(paths, lens, pl, exp, threads=4) == [True] * n
    if n <= 64:
        assert all(oracle.check_piece_hash_sync(paths, lens, pl, i, exp[20 * i:20 * i + 20]) for i in range(n))
    off = flip_offset(e)
    flip_file_byte(paths, lens, off)
    assert oracle.pool_verify_files(paths, lens, pl, exp, threads=4) == [i != off // pl for i in range(n)]
