"""One rank of the CPU test of bench.reverify_multi_leg (tests/test_bench.py).

Launched by torch.distributed.run on gloo without a GPU.  The engine's
HashPool is replaced by a CPU stand-in that verifies the rank's piece range
with the oracle (so the leg's sharding, verdict gather and timing logic run
for real); with mode "fail" the stand-in raises on rank 1's second timed
call, and every rank must then raise together rather than wait in a
collective.  Rank 0 writes {"result": ...} or {"error": ...} to argv[1].
"""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import oracle  # noqa: E402
from vortex_amd import hash_pool  # noqa: E402


class CpuPool:
    calls = 0

    def __init__(self, piece_length, device=0, **kw):
        self.pl = piece_length

    def verify_files(self, paths, lens, pl, exp, io_threads=0, first=0, count=None):
        CpuPool.calls += 1
        if MODE == "fail" and dist.get_rank() == 1 and CpuPool.calls == 3:
            raise RuntimeError("injected failure on rank 1")
        allv = oracle.pool_verify_files(paths, lens, pl, exp, threads=2)
        n = len(exp) // 20
        count = n - first if count is None else count
        return list(allv[first:first + count]), 0

    def verify_files_split(self, paths, lens, pl, exp, split, io_threads=0):
        """The engine's side of a split, on the CPU: groups of 3 pieces from
        the top of the shared claim word (the test build's take-tail hook),
        each verified with the oracle and written into the shared verdicts."""
        import ctypes

        from vortex_amd import _lib

        allv = oracle.pool_verify_files(paths, lens, pl, exp, threads=2)
        tuning = _lib.tuning()
        while True:
            was = ctypes.c_uint64()
            lo = tuning.vx_tuning_split_take_tail(ctypes.byref(split.s), 3, ctypes.byref(was))
            if lo >= was.value:
                return 0
            for i in range(lo, was.value):
                split.matched[i - split.first] = b"\x01" if allv[i] else b"\x00"

    def last_verify(self):
        return {"read_GiBps": 1.0, "copy_busy_frac": 0.5, "direct_bytes": 0}

    def close(self):
        pass


MODE = sys.argv[2] if len(sys.argv) > 2 else "ok"


def main():
    dist.init_process_group("gloo")
    hash_pool.HashPool = CpuPool  # the leg imports HashPool from vortex_amd.hash_pool at call time
    out = {}
    try:
        rm = bench.reverify_multi_leg(dist.get_rank(), dist.get_world_size(), 0, torch.device("cpu"), "gloo",
                                      True, scale=0.02, reps=2, cold_reps=1)
        out = {"result": rm}
    except RuntimeError as e:
        out = {"error": str(e)}
    if dist.get_rank() == 0:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
