#!/usr/bin/env python3
"""Where does the GPU beat vortex's own pool?  Bulk re-verify crossover grid.

For piece lengths 2/4/8/16 MiB and n_pieces 64 ... 4,096 (up to --gib GiB
per point) this times, on the same page-cache-warm file and the same host
cores:

* the engine's re-verify, vx_verify_files (pread -> pinned stages -> H2D ->
  chunk kernels -> verdicts), median of --reps calls;
* the CPU restatement of vortex's re-verify (par_iter over
  check_piece_hash_sync with SHA-NI, oracle/pool_oracle.cpp), median of 2;
* the host-only planner vx_plan_verify's predictions for both.

Then the download loop (tests/native/loop_harness: subpieces into registered
pool buffers, vx_submit on completion, drain per turn) at each piece length
for submit-to-poll latency p50/p99 against the loop's 150 ms CQE wait
(torrent.rs:42).

One torrent per point = the first n*L bytes of one synthetic file (the file
may be longer; only the torrent's bytes are read).  Every GPU verdict must be
true (expected digests from the CPU pool over an mmap of the file).  Prints
one JSON object.

usage: python tools/crossover_grid.py [--gib 8] [--reps 3] [--dir $TMPDIR]
"""
import argparse
import ctypes
import json
import mmap
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GiB = float(1 << 30)
MiB = 1 << 20


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--lens-mib", default="2,4,8,16")
    ap.add_argument("--counts", default="64,128,256,512,1024,2048,4096")
    ap.add_argument("--no-loop", action="store_true")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)

    import oracle
    from vortex_amd._lib import lib, vx_plan
    from vortex_amd.hash_pool import HashPool

    threads = max(1, min(16, len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16"))))
    size = int(a.gib * GiB) // (16 * MiB) * (16 * MiB)
    path = os.path.join(a.dir, f"vx_crossover_{os.getpid()}.bin")
    out = {"threads": threads, "file_bytes": size, "points": [], "loop": []}
    t0 = time.perf_counter()
    blk = ctypes.create_string_buffer(2 * MiB)
    try:
        with open(path, "wb") as f:
            for i in range(size // (2 * MiB)):
                oracle.lib().vxo_gen_piece(0xC055, i, 2 * MiB, 0, blk)
                f.write(blk.raw)
        out["write_s"] = round(time.perf_counter() - t0, 2)
        log("file written", out["write_s"], "s")
        fd = os.open(path, os.O_RDONLY)
        mm = mmap.mmap(fd, size, prot=mmap.PROT_READ)
        # address of the read-only mapping via numpy (ctypes cannot take a read-only buffer)
        import numpy as np

        arr = np.frombuffer(mm, dtype=np.uint8)
        addr0 = arr.ctypes.data
        for L in [int(x) * MiB for x in a.lens_mib.split(",")]:
            nmax = size // L
            ptrs = (ctypes.c_void_p * nmax)(*[addr0 + i * L for i in range(nmax)])
            lens = (ctypes.c_uint32 * nmax)(*([L] * nmax))
            dig = ctypes.create_string_buffer(20 * nmax)
            oracle.pool_verify_ptrs(ptrs, lens, nmax, None, threads, 0, None, dig)
            table = dig.raw
            with HashPool(L, slots=4, slot_bytes=512 << 20, batch_pieces=4096) as pool:
                for n in [int(x) for x in a.counts.split(",")]:
                    if n > nmax:
                        continue
                    total = n * L
                    exp = table[:20 * n]
                    pool.verify_files([path], [total], L, exp, io_threads=threads)  # warm
                    g = []
                    for _ in range(a.reps):
                        t = time.perf_counter()
                        got, bad = pool.verify_files([path], [total], L, exp, io_threads=threads)
                        g.append(time.perf_counter() - t)
                        assert all(got) and bad == 0, (L, n)
                    c = []
                    for _ in range(2):
                        t = time.perf_counter()
                        cpu = oracle.pool_verify_files([path], [total], L, exp, threads=threads)
                        c.append(time.perf_counter() - t)
                        assert all(cpu)
                    gm, cm = sorted(g)[len(g) // 2], sorted(c)[len(c) // 2]
                    p = vx_plan()
                    assert lib().vx_plan_verify(n, L, total, threads, 0.0, ctypes.byref(p)) == 0
                    pt = {"piece_MiB": L // MiB, "n": n, "GiB": round(total / GiB, 3),
                          "gpu_s": round(gm, 4), "cpu_s": round(cm, 4),
                          "gpu_GiBps": round(total / gm / GiB, 2), "cpu_GiBps": round(total / cm / GiB, 2),
                          "winner": "gpu" if gm < cm else "cpu",
                          "plan": {"gpu_s": round(p.gpu_s, 4), "cpu_s": round(p.cpu_s, 4),
                                   "chain_s": round(p.gpu_chain_s, 4), "transfer_s": round(p.gpu_transfer_s, 4),
                                   "use_gpu": p.use_gpu}}
                    out["points"].append(pt)
                    log(json.dumps(pt))
            del ptrs, lens, dig
        del arr
        mm.close()
        os.close(fd)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    if not a.no_loop:
        exe = os.path.join(ROOT, "tests", "native", "loop_harness")
        for L in [int(x) * MiB for x in a.lens_mib.split(",")]:
            n = 64
            seed = 0x5EED00CC
            exp = oracle.pool_digest_synth(seed, 0, n, L, threads=threads)
            ep = os.path.join(a.dir, f"vx_loop_exp_{os.getpid()}.bin")
            with open(ep, "wb") as f:
                f.write(exp)
            try:
                r = subprocess.run([exe, ep, str(n), str(L), str(L), hex(seed), "32", "4", "50"],
                                   capture_output=True, text=True, timeout=240)
            finally:
                os.unlink(ep)
            if r.returncode != 0:
                out["loop"].append({"piece_MiB": L // MiB, "error": r.stderr[-300:]})
                continue
            res = json.loads(r.stdout.strip().splitlines()[-1])
            p = vx_plan()
            lib().vx_plan_verify(1, L, L, threads, 0.0, ctypes.byref(p))
            res["plan_piece_latency_s"] = round(p.piece_latency_s, 4)
            res["cpu_piece_latency_s"] = round(p.cpu_piece_latency_s, 4)
            out["loop"].append(res)
            log(json.dumps(res))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
