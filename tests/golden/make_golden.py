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
