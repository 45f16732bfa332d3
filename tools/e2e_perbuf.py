#!/usr/bin/env python3
"""Host-batch e2e with vortex's buffer layout: every piece in its own
registered mmap (buf_pool.rs:92-98), so vx_verify_batch takes the chunked
gather path instead of the strided 2-D copies.  Same timing
as bench.e2e_rate (H2D + kernel + D2H of verdicts and digests).  One JSON line.

usage: python tools/e2e_perbuf.py [--pieces 1024] [--piece-len 2097152] [--chunks 0,65536]
"""
import argparse
import ctypes
import json
import mmap
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pieces", type=int, default=1024)
    ap.add_argument("--piece-len", type=int, default=2097152)
    ap.add_argument("--chunks", default="0,65536")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import oracle
    from vortex_amd._lib import check, lib
    from vortex_amd.hash_pool import HashPool

    n, pl = a.pieces, a.piece_len
    bufs = [mmap.mmap(-1, pl) for _ in range(n)]
    addrs = []
    for i, b in enumerate(bufs):
        base = ctypes.addressof(ctypes.c_char.from_buffer(b))
        oracle.lib().vxo_gen_piece(0x5EED0001, i, pl, 0, ctypes.c_void_p(base))
        addrs.append(base)
    exp = ctypes.create_string_buffer(oracle.pool_digest_synth(0x5EED0001, 0, n, pl, threads=16), 20 * n)
    ptrs = (ctypes.c_void_p * n)(*addrs)
    lens = (ctypes.c_uint32 * n)(*([pl] * n))
    matched = ctypes.create_string_buffer(n)
    digests = ctypes.create_string_buffer(20 * n)
    out = {}
    for c in [int(x) for x in a.chunks.split(",")]:
        os.environ["VX_BATCH_CHUNK"] = str(c)
        with HashPool(pl, slots=4, slot_bytes=256 << 20, batch_pieces=1024) as pool:
            for b in bufs:
                pool.register_buffer(b)
            check(lib().vx_verify_batch(pool._h, ptrs, lens, exp, min(n, 64), matched, digests), "warm")
            best = 0.0
            for _ in range(a.reps):
                t0 = time.perf_counter()
                check(lib().vx_verify_batch(pool._h, ptrs, lens, exp, n, matched, digests), "vx_verify_batch")
                best = max(best, n * pl / (time.perf_counter() - t0) / (1 << 30))
            assert matched.raw[:n] == b"\x01" * n
            rounds = int(lib().vx_tuning_chunk_rounds(pool._h))
            for b in bufs:
                pool.unregister_buffer(b)
        out[str(c)] = {"GiBps": round(best, 3), "chunk_rounds": rounds}
    print(json.dumps({"pieces": n, "piece_len": pl, "layout": "one registered mmap per piece", "results": out}))


if __name__ == "__main__":
    main()
