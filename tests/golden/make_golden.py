"""Regenerate tests/golden/*.json (run in the build container; committed output).

Independent oracles only — nothing here imports oracle/ or vortex_amd/:
  * hashlib (OpenSSL) for every digest;
  * a pure-Python restatement of the synthetic-piece spec (DESIGN.md
    "Synthetic pieces") so the C and HIP generators are pinned too;
  * the reference's implicit known answers: the pieces of
    bittorrent/src/lib.rs setup_test (169-193) and setup_seeding_test
    (256-285), rebuilt from their file contents;
  * the geometry and `pieces` table of the reference's data file
    cli/linux-mint.torrent (parsed with a minimal bencode reader; the file is
    data, only its numbers are kept).

Usage: python tests/golden/make_golden.py [/root/reference]
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
M64 = (1 << 64) - 1


def mix64(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def gen_piece(seed: int, piece: int, length: int, corrupt_every: int = 0) -> bytes:
    key = mix64(seed ^ ((piece * 0xD1B54A32D192ED03) & M64))
    out = bytearray()
    i = 0
    while len(out) < length:
        out += mix64((key + (i + 1) * 0x9E3779B97F4A7C15) & M64).to_bytes(8, "little")
        i += 1
    out = out[:length]
    if corrupt_every and length and piece % corrupt_every == corrupt_every - 1:
        out[(piece * 7919) % length] ^= 0xFF
    return bytes(out)


def pattern(n: int, salt: int = 0) -> bytes:
    return bytes(((i * 131 + 7 + salt) & 0xFF) for i in range(n))


def sha(b: bytes) -> str:
    return hashlib.sha1(b).hexdigest()


def bdecode(b: bytes, i: int = 0):
    c = b[i:i + 1]
    if c == b"i":
        j = b.index(b"e", i)
        return int(b[i + 1:j]), j + 1
    if c == b"l":
        i += 1
        out = []
        while b[i:i + 1] != b"e":
            v, i = bdecode(b, i)
            out.append(v)
        return out, i + 1
    if c == b"d":
        i += 1
        out = {}
        while b[i:i + 1] != b"e":
            k, i = bdecode(b, i)
            v, i = bdecode(b, i)
            out[k] = v
        return out, i + 1
    j = b.index(b":", i)
    n = int(b[i:j])
    return b[j + 1:j + 1 + n], j + 1 + n


def fill_bytes(fill: dict) -> bytes:
    """File contents from a fixture `fill` spec (also used by the tests)."""
    if "byte" in fill:
        return bytes([fill["byte"]]) * fill["len"]
    if "text" in fill:
        return fill["text"].encode() * fill["repeat"]
    return bytes.fromhex(fill["hex"])


def interval_segments(file_lens, pl):
    """Piece -> [(file_idx, offset_in_file, len)] by intersecting each piece's
    global byte range [p*pl, min((p+1)*pl, total)) with each file's global
    range.  A geometric statement of the mapping, independent of the
    FileStore walk (file_store.rs:126-160, 240-298) that oracle/ and the
    engine restate; zero-length intersections are omitted."""
    starts, acc = [], 0
    for L in file_lens:
        starts.append(acc)
        acc += L
    total = acc
    out = []
    for p in range((total + pl - 1) // pl):
        lo, hi = p * pl, min((p + 1) * pl, total)
        segs = []
        for fi, (s, L) in enumerate(zip(starts, file_lens)):
            a, b = max(lo, s), min(hi, s + L)
            if a < b:
                segs.append([fi, a - s, b - a])
        out.append(segs)
    return out


def interval_segments_sweep(file_lens, pl):
    """interval_segments in one O(files + pieces) sweep (same output): the
    files a piece touches are a contiguous run, so each piece starts from the
    first file that can still overlap it.  For layouts with 10^5 files."""
    starts, acc = [], 0
    for L in file_lens:
        starts.append(acc)
        acc += L
    total = acc
    out, f0 = [], 0
    for p in range((total + pl - 1) // pl):
        lo, hi = p * pl, min((p + 1) * pl, total)
        while f0 < len(file_lens) and starts[f0] + file_lens[f0] <= lo:
            f0 += 1
        segs, f = [], f0
        while f < len(file_lens) and starts[f] < hi:
            a, b = max(lo, starts[f]), min(hi, starts[f] + file_lens[f])
            if a < b:
                segs.append([f, a - starts[f], b - a])
            f += 1
        out.append(segs)
    return out


def segments_text(segs) -> str:
    """Canonical text of a segment table: one line per piece, "file offset
    length" triples joined by ';' (tests/native/segments_dump.cpp prints it)."""
    return "\n".join(";".join(f"{f} {o} {n}" for f, o, n in piece) for piece in segs) + "\n"


def many_files_lens(nfiles: int = 100_000, seed: int = 100_000):
    """A torrent of 10^5 files (not a reference layout: the scale at which a
    per-piece walk over every file, file_store.rs:238-241, turns quadratic).
    Mostly small files, 1 in 20 empty, 1 in 1,000 of 1-8 MiB."""
    import random

    r = random.Random(seed)
    out = []
    for _ in range(nfiles):
        k = r.random()
        out.append(0 if k < 0.05 else r.randrange(1 << 20, 8 << 20) if k > 0.999 else r.randrange(1, 40_000))
    return out


def many_files_layout():
    lens = many_files_lens()
    pl = 16384
    segs = interval_segments_sweep(lens, pl)
    return {"name": "many_files_100k", "source": "extra (not a reference test): tests/golden/make_golden.py "
                                                 "many_files_lens(100000, seed 100000)",
            "piece_length": pl, "nfiles": len(lens), "total": sum(lens), "num_pieces": len(segs),
            "files_sha1": hashlib.sha1(" ".join(map(str, lens)).encode()).hexdigest(),
            "segments_text_sha1": hashlib.sha1(segments_text(segs).encode()).hexdigest()}


def file_store_layouts():
    """The reference's own FileStore layout tests and integration-test
    geometries (file path order; see the fixture's `order_note`)."""
    import random

    def rnd(seed, n):
        r = random.Random(seed)
        return {"hex": bytes(r.getrandbits(8) for _ in range(n)).hex()}

    fs = "bittorrent/src/file_store.rs"
    small6 = [("f1.txt", {"byte": 1, "len": 64}), ("f2.txt", {"byte": 2, "len": 100}),
              ("f3.txt", {"byte": 3, "len": 50}), ("f4.txt", {"byte": 4, "len": 20}),
              ("f5.txt", {"byte": 5, "len": 10}), ("f6.txt", {"byte": 6, "len": 268})]
    v2 = [("f1.txt", {"byte": 1, "len": 84}), ("f2.txt", {"byte": 2, "len": 114}),
          ("f3.txt", {"byte": 3, "len": 134}), ("f4.txt", {"byte": 4, "len": 24})]
    sub, length = 32, 282
    v2_single = b"".join(bytes([i]) * sub for i in range(length // sub)) + bytes([length // sub]) * (length % sub)
    L = [
        ("basic_multifile_alinged", f"{fs}:567-576", 256,
         [(f"test/file_{i}.txt", {"byte": i, "len": 1024}) for i in range(10)]),
        ("small_multifile_misalinged", f"{fs}:578-591", 256, small6),
        ("small_multifile_misalinged_files_and_subpiece", f"{fs}:593-611 (subpiece 35)", 256, small6),
        ("multifile_not_multiple_of_piece_size", f"{fs}:613-626", 256,
         [("f1.txt", {"byte": 1, "len": 64}), ("f2.txt", {"byte": 2, "len": 256}),
          ("f3.txt", {"byte": 3, "len": 50}), ("f4.txt", {"byte": 4, "len": 20}),
          ("f5.txt", {"byte": 5, "len": 10}), ("f6.txt", {"byte": 6, "len": 300})]),
        ("multifile_misalinged_v2", f"{fs}:628-639", 64, v2),
        ("multifile_misalinged_v3", f"{fs}:641-652", 64, v2),
        ("multifile_misalinged", f"{fs}:654-663", 256,
         [(f"test/file_{i}.txt", {"byte": i, "len": 800}) for i in range(10)]),
        ("basic_single_file_aligned", f"{fs}:665-674 (random bytes; seeded here)", 256,
         [("test_single.txt", rnd(665, 1024))]),
        ("basic_single_file_aligned_unaligned_subpiece", f"{fs}:676-690 (random bytes; seeded here)", 256,
         [("test_single.txt", rnd(676, 1024))]),
        ("single_file_misaligned", f"{fs}:692-701 (random bytes; seeded here)", 256,
         [("test_single.txt", rnd(692, 1354))]),
        ("single_file_misaligned_v2", f"{fs}:703-722", 256, [("test_single.txt", {"hex": v2_single.hex()})]),
        ("disk_operations_for_all_valid_piece_indices", f"{fs}:724-760", 256,
         [("test/root/test_single.txt", {"byte": 1, "len": 10000})]),
        ("basic_seeding", "bittorrent/tests/basic_seeding.rs:27-48 (piece length 16384*8)", 16384 * 8,
         [("file2.txt", {"text": "BitTorrent Test Data!", "repeat": 200}),
          ("subdir/file3.txt", {"byte": 42, "len": 16384 * 5000 + 20000})]),
        ("chained_seeding", "bittorrent/tests/chained_seeding.rs:32-51 (piece length 16384)", 16384,
         [("file1.txt", {"text": "Chained Seeding Test!", "repeat": 150}),
          ("file2.txt", {"text": "Middle peer uploads while downloading!", "repeat": 250}),
          ("subdir/file3.txt", {"byte": 99, "len": 20480})]),
        ("pause_resume", "bittorrent/tests/pause_resume.rs:27-42 (piece length 16384)", 16384,
         [("file2.txt", {"text": "BitTorrent Test Data!", "repeat": 200}),
          ("subdir/file3.txt", {"byte": 42, "len": 16384 * 5000})]),
        # Not reference tests: edge cases of the same walk that no reference
        # test reaches (zero-length files, a file ending exactly on a piece
        # boundary, many files inside one piece, a one-byte last piece).
        ("extra_zero_length_and_boundaries", "extra (not a reference test)", 64,
         [("a", {"byte": 0xA1, "len": 64}), ("b", {"byte": 0xB2, "len": 0}), ("c", {"byte": 0xC3, "len": 3}),
          ("d", {"byte": 0xD4, "len": 0}), ("e", {"byte": 0xE5, "len": 61}), ("f", rnd(9, 130)),
          ("g", {"byte": 0x07, "len": 1}), ("h", {"byte": 0x08, "len": 1}), ("i", {"byte": 0x09, "len": 0})]),
        ("extra_many_tiny_files", "extra (not a reference test)", 1000,
         [(f"t/{k:03d}", rnd(100 + k, (k * 37) % 50)) for k in range(120)] + [("t/zz", {"byte": 1, "len": 1})]),
    ]
    out = []
    for name, src, pl, files in L:
        datas = [fill_bytes(fill) for _, fill in files]
        lens = [len(d) for d in datas]
        data = b"".join(datas)
        total = len(data)
        n = (total + pl - 1) // pl
        digests = [hashlib.sha1(data[i:i + pl]).digest() for i in range(0, total, pl)]
        ent = {"name": name, "source": src, "piece_length": pl,
               "files": [{"path": p, "len": ln, "fill": f} for (p, f), ln in zip(files, lens)],
               "total": total, "num_pieces": n, "last_piece_len": total - (n - 1) * pl if n else 0,
               "pieces_sha1_of_table": hashlib.sha1(b"".join(digests)).hexdigest()}
        if n <= 64:
            ent["pieces"] = [d.hex() for d in digests]
            ent["segments"] = interval_segments(lens, pl)
        out.append(ent)
    return out


def main(ref_root: str) -> None:
    fips = [
        {"name": "empty", "hex_input": "", "sha1": "da39a3ee5e6b4b0d3255bfef95601890afd80709"},
        {"name": "abc", "hex_input": b"abc".hex(), "sha1": "a9993e364706816aba3e25717850c26c9cd0d89d"},
        {"name": "448-bit", "hex_input": b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq".hex(),
         "sha1": "84983e441c3bd26ebaae4aa1f95129e5e54670f1"},
        {"name": "896-bit",
         "hex_input": (b"abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmno"
                       b"ijklmnopjklmnopqklmnopqrlmnopqrsmnopqrstnopqrstu").hex(),
         "sha1": "a49b2446a02c645bf419f995b67091253a04a259"},
    ]
    for v in fips:
        assert sha(bytes.fromhex(v["hex_input"])) == v["sha1"], v["name"]
    million_a = {"len": 1_000_000, "byte": 0x61, "sha1": "34aa973cd4c4daa4f61eeb2bdbad27316534016f"}
    assert sha(b"a" * 1_000_000) == million_a["sha1"]

    # Boundary lengths: every length 0..200 and the padding edges up to 4 KiB.
    lengths = list(range(0, 201)) + [247, 248, 255, 256, 257, 1000, 1023, 1024, 1025, 4095, 4096, 4097,
                                     16383, 16384, 16385, 65535, 65536, 65537]
    boundary = [{"len": n, "sha1": sha(pattern(n))} for n in lengths]

    # Reference known answers.
    sub = 16384
    setup_test = {
        "source": "bittorrent/src/lib.rs:169-193 setup_test: f3.txt = 0x03 x 16*16384, piece length 32768",
        "piece_length": 2 * sub,
        "files": [{"byte": 3, "len": 16 * sub}],
        "pieces": [sha(b"\x03" * (2 * sub))] * 8,
    }
    seeding_data = b"\x01" * 64 + b"\x02" * 100 + b"\x03" * (16 * sub)
    seeding = {
        "source": ("bittorrent/src/lib.rs:256-285 setup_seeding_test: f1=0x01x64, f2=0x02x100, "
                   "f3=0x03x262144 (files in path order), piece length 32768"),
        "piece_length": 2 * sub,
        "files": [{"byte": 1, "len": 64}, {"byte": 2, "len": 100}, {"byte": 3, "len": 16 * sub}],
        "pieces": [sha(seeding_data[i:i + 2 * sub]) for i in range(0, len(seeding_data), 2 * sub)],
    }
    assert seeding["pieces"][0] == "e620dc76973c77357d757565a36afc96d8403ae1"
    assert seeding["pieces"][8] == "2403fd426832e420b654a7cf7a035e0beaaf4cd2"
    assert setup_test["pieces"][0] == "0b5f75802398863cb57d24b30c5caa55e56062b6"

    # Synthetic generator spec, pinned by a pure-Python restatement.
    synth = []
    for seed, piece, length, ce in [(0x5EED0001, 0, 256, 0), (0x5EED0001, 1, 1000, 0), (0x5EED0002, 12345, 4096, 0),
                                    (0x5EED0002, 65535, 333, 0), (0x5EED0003, 99, 4096, 100),
                                    (0x5EED0003, 199, 4097, 100), (7, 3, 7, 4), (0x5EED0001, 2, 262144, 0)]:
        data = gen_piece(seed, piece, length, ce)
        synth.append({"seed": seed, "piece": piece, "len": length, "corrupt_every": ce,
                      "head_hex": data[:32].hex(), "sha1": sha(data)})

    out = {"fips": fips, "million_a": million_a, "boundary_pattern": "byte[i] = (i*131 + 7) & 0xff",
           "boundary": boundary, "setup_test": setup_test, "setup_seeding_test": seeding, "synthetic": synth}
    out["file_store_layouts_note"] = (
        "The reference's FileStore tests (file_store.rs:567-760) and integration tests build the torrent with "
        "lava_torrent's TorrentBuilder from a HashMap of files; the file order is the builder's, taken here as "
        "path order (the same assumption as setup_seeding_test). Tests also run each layout in reverse order, "
        "so the mapping is pinned whatever the order. `pieces` = hashlib over the concatenated files; "
        "`segments` = a geometric interval intersection (independent of the FileStore walk).")
    out["file_store_layouts"] = file_store_layouts()
    out["many_files_layout"] = many_files_layout()

    torrent_path = os.path.join(ref_root, "cli", "linux-mint.torrent")
    if os.path.exists(torrent_path):
        t, _ = bdecode(open(torrent_path, "rb").read())
        info = t[b"info"]
        pieces = info[b"pieces"]
        out["linux_mint"] = {
            "source": "cli/linux-mint.torrent (reference data file; info dict)",
            "name": info[b"name"].decode(),
            "length": info[b"length"],
            "piece_length": info[b"piece length"],
            "num_pieces": len(pieces) // 20,
            "last_piece_len": info[b"length"] - (len(pieces) // 20 - 1) * info[b"piece length"],
            "pieces_sha1_of_table": hashlib.sha1(pieces).hexdigest(),
            "first_pieces": [pieces[20 * i:20 * i + 20].hex() for i in range(4)],
        }
        with open(os.path.join(HERE, "linux_mint_pieces.bin"), "wb") as f:
            f.write(pieces)
    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "vectors.json"))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
