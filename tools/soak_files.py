#!/usr/bin/env python3
"""Soak the bulk re-verify (vx_verify_files / vx_verify_files_range) for a
fixed time: random multi-file layouts (empty files included), random piece
lengths (odd ones, ones that are not multiples of the chunk, 16 KiB-4 MiB),
flipped bytes, truncated and missing files, random piece ranges; every
call is compared with the CPU restatement oracle.pool_verify_files (test
infrastructure).  Any difference exits non-zero.  Prints one JSON line.

With --cold, every call first evicts the torrent's files from the page cache
(fsync + POSIX_FADV_DONTNEED), so the readers take their O_DIRECT path for
aligned uncached ranges (vx_files::DirectIo) and the buffered one for the
rest; the bytes read direct are summed in the JSON.  Without --dir, the soak
runs in the first disk-backed directory (bench.reverify_dir).

usage: python tools/soak_files.py [--seconds 60] [--seed 1] [--dir DIR] [--cold]
"""
import argparse
import hashlib
import json
import os
import random
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--cold", action="store_true", help="evict the files before every call")
    a = ap.parse_args()
    import bench
    import oracle
    from vortex_amd.hash_pool import HashPool

    if a.dir is None:
        a.dir = bench.reverify_dir()
    rng = random.Random(a.seed)
    t_end = time.time() + a.seconds
    stats = {"torrents": 0, "calls": 0, "pieces": 0, "bad_pieces": 0, "direct_bytes": 0, "read_bytes": 0}

    def evict(paths):
        if not a.cold:
            return
        for p in paths:
            if os.path.exists(p):
                bench.drop_cache(p)
    root = tempfile.mkdtemp(prefix="vx_soak_files_", dir=a.dir)
    try:
        while time.time() < t_end:
            pl = rng.choice([16384, 65536, 262144, 300000, (1 << 20) + 3072, 2 << 20, 4 << 20])
            nfiles = rng.randint(1, 10)
            sizes = [rng.choice([0, rng.randint(1, 4 * pl), rng.randint(1, 200), rng.randint(pl, 6 * pl),
                                 rng.randint(1, 6) * pl, rng.randint(256, 2048) * 4096])
                     for _ in range(nfiles)]
            if sum(sizes) == 0:
                sizes[0] = pl + 1
            paths = []
            for k, L in enumerate(sizes):
                p = os.path.join(root, f"f{k}.bin")
                with open(p, "wb") as f:
                    f.write(oracle.gen_piece(a.seed + stats["torrents"], k, L))
                paths.append(p)
            data = b"".join(open(p, "rb").read() for p in paths)
            exp = b"".join(hashlib.sha1(data[i:i + pl]).digest() for i in range(0, len(data), pl))
            n = len(exp) // 20
            # damage: flip a byte, truncate or remove a file
            for _ in range(rng.randint(0, 3)):
                k = rng.randrange(nfiles)
                if not os.path.exists(paths[k]):
                    continue
                cur = os.path.getsize(paths[k])  # may already be truncated
                if cur == 0:
                    continue
                what = rng.random()
                if what < 0.5:
                    with open(paths[k], "r+b") as f:
                        off = rng.randrange(cur)
                        f.seek(off)
                        b = f.read(1)
                        f.seek(off)
                        f.write(bytes([b[0] ^ 0x5A]))
                elif what < 0.8:
                    with open(paths[k], "r+b") as f:
                        f.truncate(rng.randrange(cur))
                else:
                    os.unlink(paths[k])
            want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
            slots = rng.choice([2, 3, 4])
            slot_bytes = max(pl, rng.choice([4 << 20, 32 << 20, 256 << 20]))
            with HashPool(pl, slots=slots, batch_pieces=rng.choice([4, 64, 4096]), slot_bytes=slot_bytes) as pool:
                evict(paths)
                got, bad = pool.verify_files(paths, sizes, pl, exp, io_threads=rng.choice([0, 1, 3, 8]))
                tr = pool.last_verify()
                stats["direct_bytes"] += tr["direct_bytes"]
                stats["read_bytes"] += tr["read_bytes"]
                stats["calls"] += 1
                if got != want:
                    print(json.dumps({"error": "verdicts differ", "pl": pl, "sizes": sizes}))
                    return 1
                first = rng.randrange(n)
                count = rng.randint(0, n - first)
                evict(paths)
                sub, _ = pool.verify_files(paths, sizes, pl, exp, io_threads=2, first=first, count=count)
                stats["calls"] += 1
                if sub != want[first:first + count]:
                    print(json.dumps({"error": "range verdicts differ", "pl": pl, "sizes": sizes,
                                      "first": first, "count": count}))
                    return 1
            stats["torrents"] += 1
            stats["pieces"] += n
            stats["bad_pieces"] += sum(1 for x in want if not x)
            for p in paths:
                if os.path.exists(p):
                    os.unlink(p)
            print(f"torrents {stats['torrents']}", file=sys.stderr, flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)
    print(json.dumps({"ok": True, "seconds": a.seconds, "seed": a.seed, **stats}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
