"""Helpers for the reference's FileStore layouts (tests/golden/vectors.json
`file_store_layouts`, made by tests/golden/make_golden.py from
bittorrent/src/file_store.rs:567-760 and the integration tests)."""
from __future__ import annotations

import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from make_golden import fill_bytes, interval_segments  # noqa: E402


def materialize(entry: dict, root, reverse: bool = False):
    """Write the layout's files under `root` (in fixture order, or reversed).
    Returns (paths, lens, data, expected) where data is the concatenation in
    that order and expected the n*20-byte `pieces` table of it (hashlib)."""
    files = list(entry["files"])
    if reverse:
        files = files[::-1]
    paths, lens, parts = [], [], []
    for f in files:
        p = os.path.join(str(root), f["path"])
        os.makedirs(os.path.dirname(p), exist_ok=True)
        b = fill_bytes(f["fill"])
        assert len(b) == f["len"]
        with open(p, "wb") as fh:
            fh.write(b)
        paths.append(p)
        lens.append(len(b))
        parts.append(b)
    data = b"".join(parts)
    pl = entry["piece_length"]
    expected = b"".join(hashlib.sha1(data[i:i + pl]).digest() for i in range(0, len(data), pl))
    if not reverse:
        if "pieces" in entry:
            assert [expected[20 * i:20 * i + 20].hex() for i in range(len(entry["pieces"]))] == entry["pieces"]
        assert hashlib.sha1(expected).hexdigest() == entry["pieces_sha1_of_table"]
    return paths, lens, data, expected


def flip_offset(entry: dict) -> int:
    """A deterministic byte to corrupt: 3/7 of the way in (never 0 for
    non-trivial layouts)."""
    return (entry["total"] * 3) // 7


def flip_file_byte(paths, lens, global_off: int) -> None:
    acc = 0
    for p, L in zip(paths, lens):
        if global_off < acc + L:
            with open(p, "r+b") as fh:
                fh.seek(global_off - acc)
                b = fh.read(1)
                fh.seek(global_off - acc)
                fh.write(bytes([b[0] ^ 0x5A]))
            return
        acc += L
    raise ValueError("offset past the data")


__all__ = ["materialize", "flip_offset", "flip_file_byte", "interval_segments", "fill_bytes"]
