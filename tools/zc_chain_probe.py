"""Where does the zero-copy kernel lose per block?  

On latency-bound batches the zero-copy kernel's chain ran 6-8 % slower per
block than the split kernel hashing the same pieces from HBM.  This times, on
one GPU, the same batch three ways (median of `--reps` launches, HIP events):

  split_hbm  the ragged split kernel over the pieces in HBM;
  zc_hbm     the zero-copy kernel with its sources in HBM (its own producer,
             no PCIe);
  zc_host    the zero-copy kernel reading pinned host memory (the real case);

for a few piece lengths and counts, checks that all three give the same
digests, and prints one JSON line per case with the per-block times.

    python3 tools/zc_chain_probe.py [--reps 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--loader", type=int, default=0, help="0: the zero-copy pair, 1: the three-wave form")
    a = ap.parse_args()
    import torch

    from vortex_amd import device as vdev
    from vortex_amd._lib import check, tuning

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
    hip.hipHostGetDevicePointer.restype = ctypes.c_int

    def dev_ptr(t) -> int:
        p = ctypes.c_void_p()
        assert hip.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(t.data_ptr()), 0) == 0
        return p.value

    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    for n, plen in [(32, 4 << 20), (512, 4 << 20), (32, 256 << 10), (512, 256 << 10), (8192, 256 << 10)]:
        stride = plen
        host = torch.randint(0, 256, (n * stride,), dtype=torch.uint8).pin_memory()
        hbm = host.to(dev)
        lens = torch.full((n,), plen, dtype=torch.int32, device=dev)
        offs = torch.arange(n, dtype=torch.int64, device=dev) * stride
        src_hbm = offs + hbm.data_ptr()
        src_host = offs + dev_ptr(host)  # the pinned buffer's device mapping
        digs = {k: torch.empty((n, 20), dtype=torch.uint8, device=dev) for k in ("split_hbm", "zc_hbm", "zc_host")}

        def run(kind: str) -> None:
            if kind == "split_hbm":
                vdev.sha1_ragged(hbm, offs, lens, digests=digs[kind], variant=2, validate=False)
            else:
                srcs = src_hbm if kind == "zc_hbm" else src_host
                check(tuning().vx_tuning_zero_copy_kernel(srcs.data_ptr(), lens.data_ptr(), n, digs[kind].data_ptr(),
                                                       None, None, a.loader, int(st.cuda_stream)), "zc kernel")

        res = {"pieces": n, "piece_len": plen}
        blocks = (plen + 9 + 63) // 64
        for kind in ("split_hbm", "zc_hbm", "zc_host"):
            run(kind)
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                run(kind)
                e1.record(st)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = sorted(ts)[len(ts) // 2]
            res[kind] = {"ms": round(ms, 3), "us_per_block": round(ms * 1e3 / blocks, 4),
                         "GiBps": round(n * plen / (ms * 1e-3) / (1 << 30), 2)}
        assert torch.equal(digs["split_hbm"], digs["zc_hbm"]) and torch.equal(digs["split_hbm"], digs["zc_host"])
        print(json.dumps(res), flush=True)
        del host, hbm


if __name__ == "__main__":
    main()
