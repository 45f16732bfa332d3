"""CPU: the C-ABI library builds, loads and exports every symbol the headers
declare; argument validation works without a GPU (no compute calls)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT


def declared_symbols(headers=("vx_hash.h",)):
    names = set()
    for h in headers:
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(vx_[a-z0-9_]+)\s*\(", src))
    return names


def dynamic_symbols(path):
    """Every defined dynamic symbol of a shared library (nm -D)."""
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


def test_headers_compile_as_c(tmp_path):
    c = tmp_path / "t.c"
    c.write_text('#include "vx_hash.h"\n#include "vx_synth.h"\n#include "vx_tuning.h"\nint main(void){return (int)sizeof(vx_completion) - 32;}\n')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-c", str(c),
                    "-o", str(tmp_path / "t.o")], check=True)


def test_completion_layout():
    from vortex_amd._lib import vx_completion, vx_config

    assert ctypes.sizeof(vx_completion) == 32
    assert vx_completion.digest.offset == 9
    assert ctypes.sizeof(vx_config) == 56  # ABI 3: refuse_when_full, padded to 8


def test_config_layout(tmp_path):
    """vx_config (ABI 2) as ctypes has the C struct's size and every field's
    offset: C says so, compiled here."""
    from vortex_amd._lib import CONFIG_OPTIONS, vx_config

    fields = [name for name, _ in vx_config._fields_]
    c = tmp_path / "c.c"
    body = ", ".join(f"offsetof(vx_config, {f})" for f in fields)
    c.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "vx_hash.h"\nint main(void){size_t o[] = {'
                 + body + '}; printf("%zu", sizeof(vx_config)); for (size_t i = 0; i < sizeof(o) / sizeof(o[0]); '
                 '++i) printf(" %zu", o[i]); printf("\\n"); return 0;}\n')
    exe = tmp_path / "c"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(c), "-o",
                    str(exe)], check=True)
    got = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    assert got == [ctypes.sizeof(vx_config)] + [getattr(vx_config, f).offset for f in fields]
    assert fields[5:] == list(CONFIG_OPTIONS)


def test_stats_layout(tmp_path):
    """vx_stats as ctypes (and INTEGRATION.md's VxStats, test_integration_doc)
    has the C struct's size and offsets: C says so, compiled here."""
    from vortex_amd._lib import VX_STATS_HIST, vx_stats

    c = tmp_path / "s.c"
    c.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "vx_hash.h"\nint main(void){printf("%zu %zu %zu %d\\n", '
                 'sizeof(vx_stats), offsetof(vx_stats, submit_stall_ns), offsetof(vx_stats, batch_latency_hist), '
                 'VX_STATS_HIST); return 0;}\n')
    exe = tmp_path / "s"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(c), "-o",
                    str(exe)], check=True)
    size, stall, hist, nh = map(int, subprocess.run([str(exe)], capture_output=True, text=True,
                                                     check=True).stdout.split())
    assert (size, stall, hist, nh) == (ctypes.sizeof(vx_stats), vx_stats.submit_stall_ns.offset,
                                       vx_stats.batch_latency_hist.offset, VX_STATS_HIST)


@pytest.mark.parametrize("struct,fields", [
    ("vx_verify_trace", None), ("vx_verify_round", None), ("vx_stats", ("zero_copy_slots", "zero_copy_loader_slots", "submits_refused")),
    ("vx_plan", None)])
def test_observability_layouts(tmp_path, struct, fields):
    """ABI 3's observability structs as ctypes have the C layout: size and
    every field's offset (vx_stats: the two fields ABI 3 appended)."""
    from vortex_amd import _lib

    cls = getattr(_lib, struct)
    names = list(fields or [n for n, _ in cls._fields_])
    c = tmp_path / "o.c"
    body = ", ".join(f"offsetof({struct}, {f})" for f in names)
    c.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "vx_hash.h"\nint main(void){size_t o[] = {'
                 + body + '}; printf("%zu", sizeof(' + struct + ')); for (size_t i = 0; i < sizeof(o) / sizeof(o[0]); '
                 '++i) printf(" %zu", o[i]); printf("\\n"); return 0;}\n')
    exe = tmp_path / "o"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(c), "-o",
                    str(exe)], check=True)
    got = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    assert got == [ctypes.sizeof(cls)] + [getattr(cls, f).offset for f in names]


def test_library_exports_declared_symbols(built):
    """The release library vortex links exports exactly the functions of
    vx_hash.h — no test hooks, no kernel-variant pins, no C++ internals (VERDICT
    r4 #6) — and the tuning build exports vx_hash.h + vx_tuning.h + vx_synth.h."""
    from vortex_amd import _lib

    lib = _lib.lib()
    decl = declared_symbols()
    assert decl == set(_lib.EXPORTS)
    assert dynamic_symbols(_lib.LIB_PATH) == decl
    for name in decl:
        assert hasattr(lib, name)
    assert lib.vx_abi_version() == 3 == _lib.ABI_VERSION
    tdecl = declared_symbols(("vx_tuning.h", "vx_synth.h"))
    assert tdecl == set(_lib.TUNING_EXPORTS) and not tdecl & decl
    assert dynamic_symbols(_lib.TUNING_PATH) == decl | tdecl
    assert _lib.tuning().vx_abi_version() == 3
    assert not any(n.startswith("vx_tuning") for n in dynamic_symbols(_lib.LIB_PATH))


def test_no_cpu_fallback_in_product():
    """The product path never imports or links the oracle."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "vortex_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".h", ".cpp")):
                code = [ln for ln in open(os.path.join(dirpath, f)).read().splitlines()
                        if not ln.lstrip().startswith(("//", "#", "*", "/*"))]
                text = "\n".join(code)
                assert "import oracle" not in text and "from oracle" not in text, f
                assert "liboracle" not in text and not re.search(r"\bvxo_\w+\s*\(", text), f


def test_validation_without_gpu(built):
    from vortex_amd import _lib

    L = _lib.lib()
    # argument errors are reported before anything touches a device
    assert L.vx_sha1_device_uniform(None, 64, 64, 4, None, None, None, None) == _lib.VX_EINVAL
    assert L.vx_sha1_device_uniform(ctypes.c_void_p(0x1001), 64, 64, 4, ctypes.c_void_p(0x2000), None, None,
                                    None) == _lib.VX_EINVAL  # misaligned base
    assert L.vx_sha1_device_uniform(ctypes.c_void_p(0x1000), 24, 64, 4, ctypes.c_void_p(0x2000), None, None,
                                    None) == _lib.VX_EINVAL  # stride % 16
    assert L.vx_sha1_device_uniform(ctypes.c_void_p(0x1000), 64, 64, 0, None, None, None, None) == 0  # n=0 no-op
    assert b"aligned" in L.vx_last_error() or L.vx_last_error()
    assert L.vx_strerror(_lib.VX_ERANGE) == b"piece longer than max_piece_len"
    cfg = _lib.vx_config()
    L.vx_config_default(ctypes.byref(cfg), 262144)
    assert cfg.max_piece_len == 262144 and cfg.slots >= 1 and cfg.batch_pieces >= 1
    assert cfg.slot_bytes >= 262144
    assert (cfg.zero_copy, cfg.direct_io, cfg.batch_chunk, cfg.verify_chunk, cfg.verify_cold_chunk,
            cfg.verify_ramp, cfg.refuse_when_full) == (1, 1, 65536, 0, 0, 1, 0)
    h = ctypes.c_void_p()
    # option values outside their ranges are refused before any device is looked at
    for field, value in (("zero_copy", 2), ("direct_io", 7), ("verify_ramp", 6), ("refuse_when_full", 2),
                         ("batch_chunk", 1000),
                         ("verify_chunk", 4097), ("verify_cold_chunk", 2048),
                         ("verify_chunk", 2 ** 32 - 4096), ("batch_chunk", (1 << 30) + 4096)):
        badopt = _lib.vx_config()
        L.vx_config_default(ctypes.byref(badopt), 262144)
        setattr(badopt, field, value)
        assert L.vx_create(ctypes.byref(badopt), ctypes.byref(h)) == _lib.VX_EINVAL, field
        assert field.encode() in L.vx_last_error() or b"chunk sizes" in L.vx_last_error()
    # HashPool refuses values a uint32 field would wrap (ctypes does so silently)
    from vortex_amd.hash_pool import HashPool

    for bad in (-4096, 1 << 32):
        with pytest.raises(ValueError, match="uint32"):
            HashPool(262144, verify_chunk=bad)
    if L.vx_device_count() == 0:
        assert L.vx_create(ctypes.byref(cfg), ctypes.byref(h)) == _lib.VX_ENODEV
    bad = _lib.vx_config()
    assert L.vx_create(ctypes.byref(bad), ctypes.byref(h)) == _lib.VX_EINVAL
    assert L.vx_create(None, ctypes.byref(h)) == _lib.VX_EINVAL
    # the multi-context re-verify validates its context list before any thread starts
    assert L.vx_verify_files_multi(None, 2, None, None, 0, 256, None, 0, None, 0) == _lib.VX_EINVAL
    ctxs = (ctypes.c_void_p * 2)(None, None)
    assert L.vx_verify_files_multi(ctxs, 2, None, None, 0, 256, None, 0, None, 0) == _lib.VX_EINVAL
    assert L.vx_verify_files_multi(ctxs, 0, None, None, 0, 256, None, 0, None, 0) == _lib.VX_EINVAL
    # observability entry points refuse NULL before touching anything
    st = _lib.vx_stats()
    assert L.vx_get_stats(None, ctypes.byref(st)) == _lib.VX_EINVAL
    assert L.vx_reset_stats(None) == _lib.VX_EINVAL


def test_sort_order_host_helper(built):
    import numpy as np

    from vortex_amd import _lib

    lens = np.array([5, 100, 7, 100, 0, 64], dtype=np.uint32)
    out = np.zeros_like(lens)
    assert _lib.lib().vx_sort_order(lens.ctypes.data, lens.size, out.ctypes.data) == 0
    assert out.tolist() == [1, 3, 5, 2, 0, 4]  # descending, stable


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from vortex_amd import _lib

    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(ImportError):
        _lib.lib()


def test_ragged_plan_host(built):
    """The ragged kernel planner on the BASELINE geometries:
    throughput-bound batches of equal pieces go to the lane kernel, batches
    bound by their longest chain (config 3's 4 MiB pieces, config 5's 2 MiB
    pieces, small batches) to the split kernel."""
    from vortex_amd import _lib

    plan = _lib.tuning().vx_tuning_plan_ragged
    LANE, SPLIT, WIDE = 1, 2, 5  # WIDE: split, one pair per CU (chain-bound with room to spare)
    KiB, MiB = 1024, 1 << 20
    assert plan(65536, 256 * KiB, 65536 * 256 * KiB) == LANE                     # config 2 as a ragged batch
    c3 = 262144 * 16 * KiB + 16384 * 256 * KiB + 4096 * MiB + 1024 * 4 * MiB      # config 3, 16 GiB
    assert plan(262144 + 16384 + 4096 + 1024, 4 * MiB, c3) == WIDE
    assert plan(1387, 2 * MiB, 2907832320) == WIDE                                 # config 5 geometry
    assert plan(16384, 256 * KiB, 16384 * 256 * KiB) == SPLIT                      # chip not full
    assert plan(1 << 20, 16 * KiB, (1 << 20) * 16 * KiB) == LANE                   # many short pieces


def test_zero_copy_plan_host(built):
    """The default zero-copy policy: every slot of registered
    aligned pieces is hashed from host memory whatever their length; full
    slots (>= 128 pieces) by the pair, small (latency-bound) batches by the
    three-wave form with a loader wave."""
    from vortex_amd import _lib

    zc = _lib.tuning().vx_tuning_zero_copy_plan
    KiB, MiB = 1024, 1 << 20
    assert zc(8192, 8192 * 16 * KiB) == 1       # 16 KiB pieces, a full 128 MiB slot
    assert zc(512, 512 * 256 * KiB) == 1        # config 1's 256 KiB pieces
    assert zc(512, 512 * 2 * MiB) == 1          # linux-mint's 2 MiB pieces
    assert zc(128, 128 * 4 * MiB) == 1
    assert zc(127, 127 * 16 * KiB) == 2         # a small batch from the download loop
    assert zc(32, 32 * 256 * KiB) == 2
    assert zc(1, 1) == 2


def _schedule(L, C, head, tail):
    import ctypes

    from vortex_amd import _lib

    fn = _lib.tuning().vx_tuning_chunk_schedule
    n = fn(L, C, head, tail, None, 0)
    out = (ctypes.c_uint64 * (2 * max(n, 1)))()
    assert fn(L, C, head, tail, out, n) == n
    return [(out[2 * i], out[2 * i + 1]) for i in range(n)]


def test_chunk_schedule_known(built):
    """Re-verify round boundaries at the config 5 geometry:
    2 MiB with C = 256 KiB ramps 64K, 64K, 128K, 6 x 256K, 128K, 64K, 64K."""
    KiB = 1024
    got = _schedule(2048 * KiB, 256 * KiB, 1, 1)
    assert [l // KiB for _, l in got] == [64, 64, 128] + [256] * 6 + [128, 64, 64]
    assert _schedule(2048 * KiB, 256 * KiB, 0, 0) == [(k * 256 * KiB, 256 * KiB) for k in range(8)]
    # L = 2C: head and tail ramps meet at C (round 4; before, such pieces ended on a whole-C chain)
    assert [l // KiB for _, l in _schedule(256 * KiB, 128 * KiB, 1, 1)] == [32, 32, 64, 64, 32, 32]
    # below 2C the two ramps would overlap: plain chunks
    assert _schedule(252 * KiB, 128 * KiB, 1, 1) == [(0, 128 * KiB), (128 * KiB, 124 * KiB)]
    assert _schedule(0, 256 * KiB, 1, 1) == [(0, 0)]  # an empty piece still gets its one padding round


@pytest.mark.parametrize("seed", range(3))
def test_chunk_schedule_properties(built, seed):
    """Any L, C (multiple of 4 KiB), head/tail ramp depths 0-3: rounds tile
    [0, L) in order, no round exceeds C, every boundary but L is a multiple
    of q = C / 2^(d+1) and of 64 (a non-final chunk never ends mid-block);
    with L > 2C the ramped first round is q and the ramped last round <= q."""
    import random

    rng = random.Random(seed)
    for _ in range(400):
        C = rng.choice([4096, 65536, 131072, 262144, 393216, 524288])
        L = rng.choice([rng.randrange(0, 4 * C), rng.randrange(0, 64 * C), 2 * C, 2 * C + 1, C - 1, C])
        head, tail = rng.randrange(4), rng.randrange(4)
        d = max(head, tail)
        q = C >> (d + 1)
        r = _schedule(L, C, head, tail)
        a = 0
        for off, ln in r:
            assert off == a and 0 < ln <= C or (L == 0 and (off, ln) == (0, 0))
            a += ln
            if a < L:
                assert a % 64 == 0 and (d == 0 or q < 64 or a % q == 0)
        assert a == L
        if L > 2 * C and d and q >= 64:
            assert (r[0][1] == q) == bool(head)
            if tail:
                assert r[-1][1] <= q and r[-2][1] == q
        if L > 2 * C and (d == 0 or q < 64):
            assert all(ln == C for _, ln in r[:-1])


def _plan(n, pl, total, threads=16, rate=2.0e9):
    from vortex_amd import _lib

    p = _lib.vx_plan()
    rc = _lib.lib().vx_plan_verify(n, pl, total, threads, rate, ctypes.byref(p))
    return rc, p


def _plan_g(n, pl, total, threads, g, rate=2.2e9):
    from vortex_amd import _lib

    p = _lib.vx_plan()
    assert _lib.lib().vx_plan_verify_gpus(n, pl, total, threads, rate, g, ctypes.byref(p)) == 0
    return p


def test_plan_verify_gpus_host(built):
    """vx_plan_verify_gpus (include/vx_hash.h): the bytes split over n_gpus
    links, one piece's chain unchanged.  n_gpus 0/1 is vx_plan_verify; on a
    full node (128 threads) linux-mint's 2 MiB pieces stay on the CPU pool
    whatever the GPU count (a 2 MiB chain is ~25 ms), while many short or
    many long pieces go to 8 GPUs (INTEGRATION.md "A whole node")."""
    MiB = 1 << 20
    fields = ("gpu_s", "gpu_chain_s", "gpu_transfer_s", "cpu_s", "use_gpu")
    for n, pl, total, t in ((1387, 2 * MiB, 2907832320, 16), (174, 16 * MiB, 174 * 16 * MiB, 16),
                            (11093, 256 * 1024, 11093 * 256 * 1024, 64)):
        _, base = _plan(n, pl, total, threads=t, rate=2.2e9)
        for g in (0, 1):
            q = _plan_g(n, pl, total, t, g)
            assert all(getattr(q, f) == getattr(base, f) for f in fields), (n, g)
        q8 = _plan_g(n, pl, total, t, 8)
        assert abs(q8.gpu_transfer_s * 8 - base.gpu_transfer_s) < 1e-12 and q8.gpu_chain_s == base.gpu_chain_s
        assert q8.gpu_s <= base.gpu_s and q8.cpu_s == base.cpu_s
    for g in (1, 2, 4, 8):  # full node, linux-mint: chain-bound against a 128-thread pool
        q = _plan_g(1387, 2 * MiB, 2907832320, 128, g)
        assert q.use_gpu == 0 and q.gpu_s > q.gpu_chain_s > q.cpu_s
    assert _plan_g(11093, 256 * 1024, 11093 * 256 * 1024, 64, 1).use_gpu == 0   # PCIe-bound on one link
    assert _plan_g(11093, 256 * 1024, 11093 * 256 * 1024, 64, 8).use_gpu == 1   # eight links
    assert _plan_g(8192, 16 * MiB, 8192 * 16 * MiB, 128, 1).use_gpu == 0
    assert _plan_g(8192, 16 * MiB, 8192 * 16 * MiB, 128, 8).use_gpu == 1
    from vortex_amd.hash_pool import plan_verify  # the Python mirror
    d = plan_verify(1387, 2 * MiB, 2907832320)
    assert d["use_gpu"] is True and d["gpu_s"] < d["cpu_s"]
    assert plan_verify(1387, 2 * MiB, 2907832320, cpu_threads=128, cpu_thread_rate=2.2e9, n_gpus=8)["use_gpu"] is False


def test_plan_verify_host(built):
    """vx_plan_verify, host-only: the BASELINE re-verify
    geometry goes to the GPU, a few very long pieces stay on the caller's
    pool (one lane's chain), many long pieces go back to the GPU, and a much
    larger CPU pool wins where its rate beats PCIe."""
    from vortex_amd import _lib

    MiB = 1 << 20
    rc, p = _plan(1387, 2 * MiB, 2907832320)                 # config 5 (linux-mint geometry)
    assert rc == 0 and p.use_gpu == 1
    assert p.gpu_transfer_s > p.gpu_chain_s and p.gpu_s < p.cpu_s
    rc, p = _plan(174, 16 * MiB, 174 * 16 * MiB)              # few long pieces: chain-bound
    assert rc == 0 and p.use_gpu == 0 and p.gpu_chain_s > p.gpu_transfer_s
    assert p.piece_latency_s > 0.15 > p.cpu_piece_latency_s    # past the loop's 150 ms CQE wait (torrent.rs:42)
    rc, p = _plan(8192, 16 * MiB, 8192 * 16 * MiB)            # many long pieces: PCIe-bound again
    assert rc == 0 and p.use_gpu == 1
    rc, p = _plan(8192, 16 * MiB, 8192 * 16 * MiB, threads=128)
    assert rc == 0 and p.use_gpu == 0                          # a 128-thread pool outruns PCIe
    rc, p = _plan(8192, 256 * 1024, 8192 * 256 * 1024)         # bench e2e sample
    assert rc == 0 and p.use_gpu == 1
    # the last piece may be short; n must match the total
    assert _plan(3, 1000, 2001)[0] == 0
    assert _plan(3, 1000, 3001)[0] == _lib.VX_EINVAL
    assert _plan(0, 1000, 0)[0] == 0
    assert _lib.lib().vx_plan_verify(1, 0, 1, 16, 2e9, None) == _lib.VX_EINVAL
    # monotone in the caller's pool
    prev = None
    for t in (1, 2, 4, 8, 16, 32, 64):
        cpu = _plan(4096, 4 * MiB, 4096 * 4 * MiB, threads=t)[1].cpu_s
        assert prev is None or cpu < prev
        prev = cpu


def test_plan_verify_matches_measured_grid(built):
    """The planner against the crossover grid measured on one MI355X
    (tools/crossover_grid.py -> profiles/r02/crossover/grid.json): the
    decision equals the measured winner wherever the two measured times
    differ by more than 10 % (inside that the planner keeps the CPU pool by
    design), and the predicted GPU time is within 10 % of the measured one."""
    import json

    with open(os.path.join(ROOT, "profiles", "r02", "crossover", "grid.json")) as f:
        grid = json.load(f)
    MiB = 1 << 20
    assert len(grid["points"]) >= 20
    for pt in grid["points"]:
        L = pt["piece_MiB"] * MiB
        rc, p = _plan(pt["n"], L, pt["n"] * L, threads=grid["threads"])
        assert rc == 0
        if max(pt["gpu_s"], pt["cpu_s"]) > 1.1 * min(pt["gpu_s"], pt["cpu_s"]):
            assert p.use_gpu == (pt["winner"] == "gpu"), pt
        elif pt["winner"] == "cpu":
            assert p.use_gpu == 0, pt
        assert abs(p.gpu_s / pt["gpu_s"] - 1) < 0.10, (pt, p.gpu_s)
    for lp in grid["loop"]:  # download path: latency p50 ~ one piece's chain
        rc, p = _plan(1, lp["piece_len"], lp["piece_len"])
        assert abs(p.piece_latency_s * 1e3 / lp["latency_ms_p50"] - 1) < 0.15, lp


def _gpu_test_option_values():
    """Constant values each vx_config option takes in HashPool(...) calls of the
    -m gpu tests: keyword constants, and for a keyword bound to a parametrized
    name, the constants of that parametrize list."""
    import ast

    vals = {}
    tdir = os.path.join(ROOT, "tests")
    for f in sorted(os.listdir(tdir)):
        if not (f.startswith("test_gpu") and f.endswith(".py")):
            continue
        tree = ast.parse(open(os.path.join(tdir, f)).read())
        params = {}  # parametrized name -> values, file-wide (helpers take them as arguments)
        for dec in ast.walk(tree):  # @pytest.mark.parametrize("a,b", [(..), ..])
            if isinstance(dec, ast.Call) and getattr(dec.func, "attr", "") == "parametrize" and len(dec.args) == 2:
                try:  # our own test files: constant arithmetic such as 2 << 20, no names
                    names = [x.strip() for x in ast.literal_eval(dec.args[0]).split(",")]
                    rows = eval(compile(ast.Expression(dec.args[1]), f, "eval"), {"__builtins__": {}})
                except (ValueError, NameError, TypeError):
                    continue
                for row in rows:
                    row = row if isinstance(row, tuple) else (row,)
                    for k, v in zip(names, row):
                        params.setdefault(k, set()).add(v)
        for call in ast.walk(tree):
            if isinstance(call, ast.Call) and getattr(call.func, "id", getattr(call.func, "attr", "")) == "HashPool":
                for kw in call.keywords:
                    if isinstance(kw.value, ast.Constant):
                        vals.setdefault(kw.arg, set()).add(kw.value.value)
                    elif isinstance(kw.value, ast.Name) and kw.value.id in params:
                        vals.setdefault(kw.arg, set()).update(params[kw.value.id])
                    elif kw.arg is None and isinstance(kw.value, ast.Name):  # **opts built from a parametrized name
                        for name, vs in params.items():
                            for v in vs:
                                vals.setdefault(f"**{kw.value.id}", set()).add((name, v))
    return vals


def test_every_engine_option_is_tested_off_default(built):
    """The engine takes its configuration from vx_config only:
    no getenv anywhere in the product library's sources, and every ABI-2
    option is exercised by some -m gpu test at a value other than
    vx_config_default's (and so checked against the oracle there)."""
    from vortex_amd import _lib

    csrc = os.path.join(ROOT, "vortex_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".hpp", ".h", ".cpp", ".inc")):
            text = open(os.path.join(csrc, f)).read()
            assert not re.search(r"\bgetenv\s*\(|secure_getenv|environ\b", text), f
    for f in os.listdir(os.path.join(ROOT, "vortex_amd")):
        if f.endswith(".py"):
            text = open(os.path.join(ROOT, "vortex_amd", f)).read()
            assert "os.environ.get(\"VX_" not in text and "getenv(\"VX_" not in text, f
    cfg = _lib.vx_config()
    _lib.lib().vx_config_default(ctypes.byref(cfg), 262144)
    vals = _gpu_test_option_values()
    # **opts dicts: {"batch_chunk": chunk} with chunk parametrized
    for key, pairs in vals.items():
        if key.startswith("**"):
            for name, v in pairs:
                if name == "chunk" and v is not None:
                    vals.setdefault("batch_chunk", set()).add(v)
    for opt in _lib.CONFIG_OPTIONS:
        default = getattr(cfg, opt)
        tested = {v for v in vals.get(opt, set()) if isinstance(v, int)}
        assert tested - {default}, f"vx_config.{opt}: no -m gpu test sets a non-default value (seen {tested})"


def _split(n, pl, total, threads, rate=2.2e9, g=1):
    from vortex_amd import _lib

    p = _lib.vx_plan()
    first, count = ctypes.c_uint64(), ctypes.c_uint64()
    assert _lib.lib().vx_plan_verify_split(n, pl, total, threads, rate, g, ctypes.byref(first), ctypes.byref(count),
                                           ctypes.byref(p)) == 0
    return first.value, count.value, p


def test_plan_verify_split_host(built):
    """vx_plan_verify_split (include/vx_hash.h), host-only: the GPUs take a
    contiguous tail, the pool the head, and the split's predicted time —
    the slower side's — never exceeds either side alone; it keeps the pool
    alone (count 0) when no split beats it by the 10 % margin, e.g. linux-mint
    on a full 128-thread node, where one 2 MiB chain (~25 ms) outlasts the
    whole pool (~11 ms)."""
    MiB = 1 << 20
    for n, pl, total, t, g in ((1387, 2 * MiB, 2907832320, 16, 1), (11093, 256 * 1024, 11093 * 256 * 1024, 64, 1),
                               (174, 16 * MiB, 174 * 16 * MiB, 16, 1), (8192, 16 * MiB, 8192 * 16 * MiB, 128, 8),
                               (65536, 256 * 1024, 65536 * 256 * 1024, 16, 1), (3, 4 * MiB, 3 * 4 * MiB, 16, 1)):
        first, count, p = _split(n, pl, total, t, g=g)
        assert first + count == n and 0 <= count <= n
        alone_cpu = _plan_g(n, pl, total, t, g).cpu_s
        alone_gpu = _plan_g(n, pl, total, t, g).gpu_s
        t_split = max(p.gpu_s, p.cpu_s)
        if count:
            assert p.use_gpu == 1 and t_split * 1.1 < alone_cpu and t_split <= alone_gpu * 1.0001, (n, pl, t)
            assert p.gpu_s > 0 and (count == n or p.cpu_s > 0)
        else:
            assert p.use_gpu == 0 and p.gpu_s == 0 and p.cpu_s == pytest.approx(alone_cpu)
    # config 5 beside a 12-thread pool (the box's 16 threads less the engine's 8 readers' share): the
    # GPU takes most pieces and the two sides meet; measured: 763 pieces on the GPU gave 38 / 48 ms
    # (GPU / pool side), 892 the best of three points on two boxes (profiles/r05/split/), and 944
    # the best on four HEAD bench runs, 55.6-57.8 GiB/s (refit_r05_bench.json)
    first, count, p = _split(1387, 2 * MiB, 2907832320, 12, rate=2.32e9)
    assert 800 < count < 950 and abs(p.gpu_s - p.cpu_s) < 0.15 * max(p.gpu_s, p.cpu_s)
    assert 2907832320 / max(p.gpu_s, p.cpu_s) / (1 << 30) == pytest.approx(57, rel=0.1)
    # and the split is below the GPU alone (measured 15-30 % on the box)
    assert max(p.gpu_s, p.cpu_s) < 0.9 * _plan_g(1387, 2 * MiB, 2907832320, 16, 1).gpu_s
    # full node: pool alone
    assert _split(1387, 2 * MiB, 2907832320, 128, g=8)[1] == 0
    # one piece and an empty torrent
    assert _split(1, 2 * MiB, 2 * MiB, 16)[1] == 0 and _split(0, 2 * MiB, 0, 16)[:2] == (0, 0)
    from vortex_amd import _lib
    assert _lib.lib().vx_plan_verify_split(10, 0, 10, 16, 2e9, 1, None, None, None) == _lib.VX_EINVAL
    from vortex_amd.hash_pool import plan_verify_split
    d = plan_verify_split(1387, 2 * MiB, 2907832320, cpu_threads=12, cpu_thread_rate=2.32e9)
    assert (d["gpu_first"], d["gpu_count"]) == (first, count) and d["use_gpu"] is True


def test_plan_verify_split_on_measured_grid(built):
    """Against the measured crossover grid (profiles/r02/crossover/grid.json,
    GPU and CPU-pool times of the same warm files on one box): wherever the
    split takes part, the two sides' measured rates put through the split's
    proportions predict a call no slower than the faster side alone."""
    import json

    grid = json.load(open(os.path.join(ROOT, "profiles", "r02", "crossover", "grid.json")))
    threads = grid["threads"]
    seen = 0
    for pt in grid["points"]:
        n, L = pt["n"], pt["piece_MiB"] << 20
        g_s, c_s = pt["gpu_s"], pt["cpu_s"]
        first, count, p = _split(n, L, n * L, threads, rate=n * L / c_s / threads)
        if not count:
            continue
        seen += 1
        # measured rates, each side on its share (the GPU side keeps its fixed chain floor)
        gpu_side = max(g_s * count / n, p.gpu_chain_s)
        cpu_side = c_s * first / n
        assert max(gpu_side, cpu_side) <= min(g_s, c_s) * 1.0001, pt
    assert seen >= 5


def test_plan_verify_decisions_on_the_round5_grid(built):
    """The same decisions on the crossover grid re-measured on round 5's engine
    (profiles/r05/crossover/grid.json, another box): wherever the measured GPU
    and CPU-pool times differ by more than 10 % the planner picks the measured
    winner, and the chain-bound points (the GPU side's floor) are predicted
    within 10 %."""
    import json

    with open(os.path.join(ROOT, "profiles", "r05", "crossover", "grid.json")) as f:
        grid = json.load(f)
    MiB = 1 << 20
    assert len(grid["points"]) >= 20
    for pt in grid["points"]:
        L = pt["piece_MiB"] * MiB
        rc, p = _plan(pt["n"], L, pt["n"] * L, threads=grid["threads"])
        assert rc == 0
        if max(pt["gpu_s"], pt["cpu_s"]) > 1.1 * min(pt["gpu_s"], pt["cpu_s"]):
            assert p.use_gpu == (pt["winner"] == "gpu"), pt
        if pt["n"] <= 256:  # chain-bound: one lane's chain, whatever the host
            assert abs(p.gpu_s / pt["gpu_s"] - 1) < 0.10, (pt, p.gpu_s)


def _split_scan(n, pl, total, threads, rate, g):
    """Every split point scored by the model of DESIGN.md §6.6 (the scan the
    engine replaced with a bisection): the GPU side at 0.74 of the
    link beside the pool, the pool at 0.80 of its rate beside the engine."""
    import math

    chain_block, pcie, setup, loss, margin = 0.76e-6, 52.0 * (1 << 30), 1.5e-3, 0.08, 1.1
    last = total - (n - 1) * pl if n else 0

    def gpu(k):
        b = (k - 1) * pl + last
        ch = math.ceil((pl + 9) / 64) * chain_block
        tr = b / (pcie * (0.74 if k < n else 1.0)) / max(1, g)
        return max(tr, ch) + setup + loss * min(tr, ch)

    def cpu(k):
        if k >= n:
            return 0.0
        return math.ceil((n - k) / threads) * (pl / (rate * 0.80 if k else rate))

    best_k, best_t = 0, cpu(0)
    for k in range(1, n + 1):
        t = max(gpu(k), cpu(k))
        if t < best_t:
            best_k, best_t = k, t
    if best_k and best_t * margin >= cpu(0):
        best_k = 0
    return best_k


@pytest.mark.parametrize("n,pl,threads,rate,g", [(1387, 2 << 20, 12, 2.32e9, 1), (1387, 2 << 20, 16, 2.2e9, 1),
                                                 (11093, 256 << 10, 64, 2.2e9, 1), (4000, 1 << 20, 8, 1.5e9, 2),
                                                 (20000, 16 << 10, 16, 2.2e9, 1), (700, 8 << 20, 24, 2.0e9, 4),
                                                 (1387, 2 << 20, 128, 2.2e9, 8), (2, 4 << 20, 1, 2.0e9, 1)])
def test_plan_verify_split_bisection_matches_scan(built, n, pl, threads, rate, g):
    """The bisected planner picks the point the exhaustive scan of the same
    model picks (the last piece shorter, so the sides' times are not
    symmetric)."""
    total = n * pl - pl // 3
    first, count, _ = _split(n, pl, total, threads, rate=rate, g=g)
    assert count == _split_scan(n, pl, total, threads, rate, g), (first, count)


def test_plan_verify_split_is_fast_on_huge_torrents(built):
    """A multi-TB torrent of 16 KiB pieces (10^8 pieces): the planner answers
    in well under a millisecond per call (it used to score every split point)."""
    import time

    n, pl = 100_000_000, 16 << 10
    t0 = time.perf_counter()
    for _ in range(10):
        first, count, p = _split(n, pl, n * pl, 16)
    assert (time.perf_counter() - t0) / 10 < 0.005
    assert first + count == n
