"""Can the hash kernels read registered host memory themselves?  

The async path moves each slot's pieces with a gather kernel into HBM and then
hashes them, one after the other on the slot's stream.  If the hash kernel's
own loads could pull the pieces over PCIe at the copy rate, a slot would take
max(transfer, chain) instead of transfer + chain.  This probe points the
existing uniform kernels (split at <= 16,384 pieces, lane above, or pinned
with `variant`) at pinned host memory through its device mapping
(hipHostGetDevicePointer) and compares, on one GPU:

  * the same batch device-resident (kernel time),
  * zero-copy from pinned host memory, one stream and `--streams` batches on
    concurrent streams (the async slots),
  * a plain pinned H2D copy of the same bytes,

and checks that the zero-copy digests equal the device-resident ones.
One JSON line per case.

    python3 tools/zero_copy_probe.py [--pieces 512] [--len 262144] [--streams 4]
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
    ap.add_argument("--pieces", type=int, default=512)
    ap.add_argument("--len", type=int, default=262144)
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="0,1,2")
    a = ap.parse_args()

    import torch

    from vortex_amd._lib import check, lib

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
    hip.hipHostGetDevicePointer.restype = ctypes.c_int

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n, L, S = a.pieces, a.len, a.streams
    stride = (L + 255) // 256 * 256
    nbytes = n * stride
    GiB = float(1 << 30)

    host = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8).pin_memory() for _ in range(S)]
    dptr = []
    for h in host:
        p = ctypes.c_void_p()
        rc = hip.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(h.data_ptr()), 0)
        assert rc == 0, f"hipHostGetDevicePointer failed: {rc}"
        dptr.append(p.value)
    resident = [h.to(dev) for h in host]
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    dig_res = [torch.empty((n, 20), dtype=torch.uint8, device=dev) for _ in range(S)]
    dig_zc = [torch.empty((n, 20), dtype=torch.uint8, device=dev) for _ in range(S)]

    def launch(base: int, dig: torch.Tensor, st: torch.cuda.Stream, variant: int) -> None:
        rc = lib().vx_sha1_device_uniform_variant(base, stride, L, n, dig.data_ptr(), None, None,
                                                   int(st.cuda_stream), variant)
        check(rc, "vx_sha1_device_uniform_variant")

    def timed(fn, k: int) -> float:
        """Wall ms of fn() over k concurrent streams (events on each)."""
        torch.cuda.synchronize()
        e0 = [torch.cuda.Event(enable_timing=True) for _ in range(k)]
        e1 = [torch.cuda.Event(enable_timing=True) for _ in range(k)]
        for j in range(k):
            e0[j].record(streams[j])
        fn(k)
        for j in range(k):
            e1[j].record(streams[j])
        torch.cuda.synchronize()
        start = min(range(k), key=lambda j: 0)
        return max(e0[start].elapsed_time(e1[j]) for j in range(k))

    out = []
    for variant in [int(v) for v in a.variants.split(",")]:
        for k in sorted({1, S}):
            for name, src in (("resident", [r.data_ptr() for r in resident]), ("zero_copy", dptr)):
                digs = dig_res if name == "resident" else dig_zc

                def go(kk: int) -> None:
                    for j in range(kk):
                        launch(src[j], digs[j], streams[j], variant)

                timed(go, k)  # warm-up
                runs = [timed(go, k) for _ in range(a.reps)]
                ms = sorted(runs)[len(runs) // 2]
                rec = {"case": name, "variant": variant, "streams": k, "pieces": n, "len": L,
                       "ms_median": round(ms, 3), "ms_runs": [round(x, 3) for x in runs],
                       "GiBps": round(k * n * L / (ms * 1e-3) / GiB, 2)}
                print(json.dumps(rec), flush=True)
                out.append(rec)
            for j in range(k):
                assert torch.equal(dig_res[j], dig_zc[j]), f"variant {variant}: zero-copy digests differ (stream {j})"
    # plain pinned H2D copy of the same bytes, one stream
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    runs = []
    for _ in range(a.reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dst.copy_(host[0], non_blocking=True)
        e1.record()
        torch.cuda.synchronize()
        runs.append(e0.elapsed_time(e1))
    ms = sorted(runs[1:])[len(runs[1:]) // 2]
    print(json.dumps({"case": "h2d_copy", "bytes": nbytes, "ms_median": round(ms, 3),
                      "GiBps": round(nbytes / (ms * 1e-3) / GiB, 2)}), flush=True)


if __name__ == "__main__":
    main()
