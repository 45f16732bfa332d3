#!/usr/bin/env python3
"""A/B of the config-5 re-verify pipeline, warm and cold.

Writes the linux-mint-geometry file once (fsync'd, on a disk-backed
filesystem: bench.reverify_dir), then for every engine configuration
(vx_config options, vortex_amd._lib.CONFIG_OPTIONS) runs `--reps` warm calls and `--cold-reps` calls
after evicting the file (fsync + POSIX_FADV_DONTNEED), alternating
configurations per rep so box drift hits all of them alike.  Prints one JSON
line per configuration with the GiB/s runs and each call's
vx_tuning_last_verify budget, and the CPU pool on the same file.

usage: python tools/reverify_ab.py [--reps 3] [--cold-reps 2] [--configs name=K=V,K=V;...]
e.g. --configs "default=;cold1m=verify_cold_chunk=1048576;buffered=direct_io=0".
A configuration's IO_THREADS=N sets its io_threads (default: the process's CPU
share), SLOTS=N / SLOT_MIB=M its slot count and size (default 4 x 512 MiB).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = "default=;buffered=direct_io=0"


def parse(spec):
    out = []
    for item in spec.split(";"):
        name, _, kv = item.partition("=")
        opts = dict(p.split("=", 1) for p in kv.split(",") if p)
        out.append((name, opts))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cold-reps", type=int, default=2)
    ap.add_argument("--configs", default=DEFAULT)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cold-only", action="store_true")
    a = ap.parse_args()
    import ctypes

    import torch  # noqa: F401  (one HIP runtime)

    import bench
    import oracle
    from vortex_amd.hash_pool import HashPool

    pl, total = 2097152, 2907832320
    n = (total + pl - 1) // pl
    last = total - (n - 1) * pl
    threads = bench.cpu_share()
    d = bench.reverify_dir()
    path = os.path.join(d, f"vx_ab_linuxmint_{os.getpid()}.iso")
    buf = ctypes.create_string_buffer(pl)
    configs = parse(a.configs)
    io = {name: int(opts.pop("IO_THREADS", 0)) or threads for name, opts in configs}
    geom = {name: (int(opts.pop("SLOTS", 4)), int(opts.pop("SLOT_MIB", 512))) for name, opts in configs}
    res = {name: {"warm": [], "cold": [], "warm_tr": [], "cold_tr": [], "options": opts, "io_threads": io[name]}
           for name, opts in configs}
    cpu = {"warm": [], "cold": []}
    try:
        with open(path, "wb") as f:
            for i in range(n):
                L = last if i == n - 1 else pl
                oracle.lib().vxo_gen_piece(0x5EED0005, i, L, 0, buf)
                f.write(memoryview(buf)[:L])
            f.flush()
            os.fsync(f.fileno())
        exp = oracle.pool_digest_synth(0x5EED0005, 0, n, pl, last_index=n - 1, last_len=last, threads=threads)
        cache_nodes = page_cache_nodes(path)
        pools = {}
        for name, opts in configs:
            pools[name] = HashPool(pl, slots=geom[name][0], slot_bytes=geom[name][1] << 20, batch_pieces=4096,
                                   **{k: int(v, 0) for k, v in opts.items()})
            got, bad = pools[name].verify_files([path], [total], pl, exp, io_threads=io[name])  # warm-up
            assert all(got) and bad == 0
        for leg, reps in (("warm", 0 if a.cold_only else a.reps), ("cold", a.cold_reps)):
            for _ in range(reps):
                for name, _env in configs:
                    if leg == "cold":
                        bench.drop_cache(path)
                    t0 = time.perf_counter()
                    got, bad = pools[name].verify_files([path], [total], pl, exp, io_threads=io[name])
                    el = time.perf_counter() - t0
                    assert all(got) and bad == 0
                    res[name][leg].append(round(total / el / (1 << 30), 2))
                    tr = pools[name].last_verify()
                    res[name][leg + "_tr"].append({k: (round(v, 3) if isinstance(v, float) else v)
                                                   for k, v in tr.items()})
                    print(f"{leg} {name}: {res[name][leg][-1]} GiB/s", file=sys.stderr, flush=True)
                if not a.no_cpu:
                    if leg == "cold":
                        bench.drop_cache(path)
                    t0 = time.perf_counter()
                    ok = oracle.pool_verify_files([path], [total], pl, exp, threads=threads)
                    cpu[leg].append(round(total / (time.perf_counter() - t0) / (1 << 30), 2))
                    assert all(ok)
        for p in pools.values():
            p.close()
    finally:
        if os.path.exists(path):
            os.unlink(path)
    for name, _ in configs:
        print(json.dumps({"config": name, **res[name]}))
    node = None
    try:
        pr = torch.cuda.get_device_properties(0)
        bus = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        node = open(f"/sys/bus/pci/devices/{bus}/numa_node").read().strip()
    except Exception as e:  # noqa: BLE001  (diagnostic only)
        node = f"? ({e})"
    print(json.dumps({"config": "cpu_pool", "threads": threads, **cpu, "dir": d, "fs": bench.fs_type(d),
                      "gpu_numa_node": node, "page_cache_pages_by_node": cache_nodes}))


def page_cache_nodes(path, samples=4096):
    """NUMA node of a sample of the file's page-cache pages: map the file,
    touch one byte per sampled page (a minor fault maps the cached page, no
    copy) and ask move_pages(2) with nodes=NULL where each page lives."""
    import ctypes
    import mmap as _mmap

    libc = ctypes.CDLL(None, use_errno=True)
    size = os.path.getsize(path)
    page = _mmap.PAGESIZE
    with open(path, "rb") as f:
        m = _mmap.mmap(f.fileno(), size, prot=_mmap.PROT_READ)
        try:
            import numpy as np

            mv = memoryview(m)
            a = np.frombuffer(mv, dtype=np.uint8)  # the mapping's address via the buffer protocol
            start = a.ctypes.data
            step = max(1, (size // page) // samples)
            idx = list(range(0, size // page, step))
            for i in idx:
                _ = int(a[i * page])  # map the page
            ptrs = (ctypes.c_void_p * len(idx))(*[start + i * page for i in idx])
            status = (ctypes.c_int * len(idx))()
            SYS_move_pages = 279  # x86_64
            rc = libc.syscall(SYS_move_pages, 0, ctypes.c_ulong(len(idx)), ptrs, None, status, 0)
            out = {}
            if rc == 0:
                for st in status:
                    k = f"N{st}" if st >= 0 else f"err{-st}"
                    out[k] = out.get(k, 0) + 1
            else:
                out["error"] = ctypes.get_errno()
            del a, mv
            return out
        finally:
            m.close()


if __name__ == "__main__":
    main()
