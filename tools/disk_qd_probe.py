"""How deep must the re-verify's O_DIRECT reads queue to saturate the GPU
box's disk?  (cold config 5.)

The engine's cold re-verify keeps one synchronous read per reader thread in
flight (16 readers = queue depth 16) and reached 11-18 GiB/s.  This probe
reads one evicted 3 GiB file with O_DIRECT at several thread counts (= queue
depths) and block sizes, interleaved per repetition, and prints one JSON line
per point.  Threads block in the kernel during a direct read, so the box's
16-CPU quota does not bound them.

    python3 tools/disk_qd_probe.py [--dir /var/tmp] [--gib 3] [--reps 2]
"""
from __future__ import annotations

import argparse
import json
import mmap
import os
import time
from concurrent.futures import ThreadPoolExecutor


def drop(path: str) -> None:
    fd = os.open(path, os.O_RDONLY)
    os.fsync(fd)
    os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
    os.close(fd)


def run(path: str, size: int, bs: int, threads: int, direct: bool) -> float:
    drop(path)
    fd = os.open(path, os.O_RDONLY | (os.O_DIRECT if direct else 0))
    n = size // bs

    def work(t: int) -> int:
        buf = mmap.mmap(-1, bs)  # page-aligned, as O_DIRECT needs
        got = 0
        for i in range(t, n, threads):
            got += os.preadv(fd, [buf], i * bs)
        return got

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        tot = sum(ex.map(work, range(threads)))
    el = time.perf_counter() - t0
    os.close(fd)
    assert tot == n * bs
    return tot / el / 2**30


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/var/tmp")
    ap.add_argument("--gib", type=float, default=3.0)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--threads", default="8,16,32,64,128")
    ap.add_argument("--bs", default="262144,1048576")
    args = ap.parse_args()
    path = os.path.join(args.dir, f"vx_qd_probe_{os.getpid()}.bin")
    size = int(args.gib * 2**30) // (1 << 20) * (1 << 20)
    chunk = os.urandom(64 << 20)
    t0 = time.perf_counter()
    with open(path, "wb") as f:
        for _ in range(size // len(chunk)):
            f.write(chunk)
        f.write(chunk[: size % len(chunk)])
        f.flush()
        os.fsync(f.fileno())
    print(json.dumps({"file": path, "bytes": size, "write_s": round(time.perf_counter() - t0, 2)}), flush=True)
    try:
        threads = [int(x) for x in args.threads.split(",")]
        sizes = [int(x) for x in args.bs.split(",")]
        for rep in range(args.reps):
            for bs in sizes:
                for th in threads:
                    r = run(path, size, bs, th, True)
                    print(json.dumps({"rep": rep, "direct": True, "bs": bs, "threads": th, "GiBps": round(r, 2)}),
                          flush=True)
            r = run(path, size, 1 << 20, 16, False)
            print(json.dumps({"rep": rep, "direct": False, "bs": 1 << 20, "threads": 16, "GiBps": round(r, 2)}),
                  flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
