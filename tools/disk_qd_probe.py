"""How deep must the re-verify's O_DIRECT reads queue to saturate the GPU
box's disk?  (cold config 5.)

The engine's cold re-verify keeps one synchronous read per reader thread in
flight (16 readers = queue depth 16) and reached 11-18 GiB/s.  This probe
reads one evicted 3 GiB file with O_DIRECT at several thread counts (= queue
depths) and block sizes, interleaved per repetition, and prints one JSON line
per point.  Threads block in the kernel during a direct read, so the box's
16-CPU quota does not bound them.

    python3 tools/disk_qd_probe.py [--dir /var/tmp] [--gib 3] [--reps 2] [--piece 2097152]
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


def run(path: str, size: int, bs: int, threads: int, direct: bool, piece: int = 0, spread: str = "") -> float:
    """piece = 0: blocks in file order, thread t taking every threads-th one.
    piece > 0: the chunk rounds' order: round k reads bytes
    [k*bs, (k+1)*bs) of every piece-byte piece, rounds one after another.
    spread: "" = each thread reads into one reused bs buffer; "4k" / "huge" =
    every block lands at its own file offset in one file-sized buffer (as the
    engine's stages spread reads over GBs), huge with MADV_HUGEPAGE; "<N>m" /
    "<N>g" = at its file offset modulo an N MiB / GiB buffer."""
    drop(path)
    fd = os.open(path, os.O_RDONLY | (os.O_DIRECT if direct else 0))
    if piece:
        offs = [i * piece + k * bs for k in range(piece // bs) for i in range(size // piece)]
    else:
        offs = [i * bs for i in range(size // bs)]

    big = None
    foot = size
    if spread:
        if spread[-1] in "mg":  # a footprint: destinations wrap around the first N MiB / GiB
            foot = min(size, int(spread[:-1]) << (20 if spread[-1] == "m" else 30))
        big = mmap.mmap(-1, foot)
        if spread == "huge":
            big.madvise(mmap.MADV_HUGEPAGE)
        big.write(bytes(foot))  # fault every page in before the clock starts
        view = memoryview(big)

    def work(t: int) -> int:
        buf = mmap.mmap(-1, bs)  # page-aligned, as O_DIRECT needs
        got = 0
        for o in offs[t::threads]:
            d = o % foot
            got += os.preadv(fd, [view[d:d + bs] if big is not None else buf], o)
        return got

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        tot = sum(ex.map(work, range(threads)))
    el = time.perf_counter() - t0
    os.close(fd)
    assert tot == len(offs) * bs
    if big is not None:
        view.release()
        big.close()
    return tot / el / 2**30


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/var/tmp")
    ap.add_argument("--gib", type=float, default=3.0)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--threads", default="8,16,32,64,128")
    ap.add_argument("--bs", default="262144,1048576")
    ap.add_argument("--piece", type=int, default=0, help="also read in the chunk rounds' order over pieces of this size")
    ap.add_argument("--spread", default="", help="comma list of destination layouts to add: 4k, huge")
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
                    for pc in ([0, args.piece] if args.piece else [0]):
                        for sp in [""] + [x for x in args.spread.split(",") if x]:
                            r = run(path, size, bs, th, True, pc, sp)
                            print(json.dumps({"rep": rep, "direct": True, "bs": bs, "threads": th, "piece": pc,
                                              "spread": sp, "GiBps": round(r, 2)}), flush=True)
            r = run(path, size, 1 << 20, 16, False)
            print(json.dumps({"rep": rep, "direct": False, "bs": 1 << 20, "threads": 16, "GiBps": round(r, 2)}),
                  flush=True)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
