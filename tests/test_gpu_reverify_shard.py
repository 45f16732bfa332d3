"""GPU: one rank's shard of the bulk re-verify (vx_verify_files_range) and the
multi-rank re-verify (shard.verify_files_sharded: each rank verifies its piece
range on its GPU, verdicts all-gathered), against the oracle's restatement of
torrent.rs:716-761 / file_store.rs:228-303 over the same files."""
import hashlib
import json
import os
import socket
import subprocess
import sys

import pytest

import oracle
from conftest import ROOT

pytestmark = pytest.mark.gpu


def _torrent(tmp_path, pl, sizes, seed):
    paths = []
    for k, L in enumerate(sizes):
        p = tmp_path / f"r{k}.bin"
        p.write_bytes(oracle.gen_piece(seed, k, L))
        paths.append(str(p))
    data = b"".join(open(p, "rb").read() for p in paths)
    exp = b"".join(hashlib.sha1(data[i:i + pl]).digest() for i in range(0, len(data), pl))
    return paths, exp


def _damage(paths, pl):
    with open(paths[2], "r+b") as f:  # flip one byte
        f.seek(pl + 3)
        b = f.read(1)
        f.seek(pl + 3)
        f.write(bytes([b[0] ^ 0x40]))
    with open(paths[4], "r+b") as f:
        f.truncate(pl // 3)
    os.unlink(paths[5])


@pytest.mark.parametrize("pl", [256 * 1024, 1 << 20])  # whole-piece path, chunked path
def test_verify_files_range(built, gpu, tmp_path, pl):
    from vortex_amd._lib import VX_EINVAL, VxError
    from vortex_amd.hash_pool import HashPool

    sizes = [3, 4 * pl + 17, 2 * pl, 0, 3 * pl - 5, pl + 1, 64, 2 * pl + pl // 2]
    paths, exp = _torrent(tmp_path, pl, sizes, 21)
    n = len(exp) // 20
    _damage(paths, pl)
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    assert not all(want) and any(want)
    with HashPool(pl, slots=3, batch_pieces=4, slot_bytes=3 << 20) as pool:
        full, bad_full = pool.verify_files(paths, sizes, pl, exp, io_threads=3)
        assert full == want
        total_bad = 0
        for first, count in [(0, n), (0, 1), (n - 1, 1), (3, 5), (n // 2, n - n // 2), (7, 0), (n, 0)]:
            got, bad = pool.verify_files(paths, sizes, pl, exp, io_threads=3, first=first, count=count)
            assert got == want[first:first + count], (first, count)
            assert 0 <= bad <= count
        # a partition of [0, n) finds every I/O-error piece exactly once
        for first in range(0, n, 3):
            total_bad += pool.verify_files(paths, sizes, pl, exp, first=first, count=min(3, n - first))[1]
        assert total_bad == bad_full
        for first, count in [(n, 1), (n - 1, 2), (n + 5, 0)]:
            with pytest.raises(VxError) as e:
                pool.verify_files(paths, sizes, pl, exp, first=first, count=count)
            assert e.value.code == VX_EINVAL


@pytest.mark.parametrize("pl", [256 * 1024, 1 << 20])
def test_split_verify_with_the_pool(built, gpu, tmp_path, pl):
    """The split re-verify (INTEGRATION.md "The split", bench.py reverify.split):
    the engine verifies the tail [first, n) with vx_verify_files_range while
    the CPU pool restatement (vortex's par_iter stand-in) verifies the head
    [0, first), both at once on one damaged multi-file torrent; the merged
    verdicts equal the pool's over the whole torrent at every split point,
    and vx_plan_verify_split's point lies in range."""
    sys.path.insert(0, ROOT)
    import bench
    from vortex_amd.hash_pool import HashPool, plan_verify_split

    sizes = [3, 4 * pl + 17, 2 * pl, 0, 3 * pl - 5, pl + 1, 64, 2 * pl + pl // 2]
    paths, exp = _torrent(tmp_path, pl, sizes, 23)
    n = len(exp) // 20
    _damage(paths, pl)
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    plan = plan_verify_split(n, pl, sum(sizes), cpu_threads=4)
    assert plan["gpu_first"] + plan["gpu_count"] == n
    with HashPool(pl, slots=3, batch_pieces=4, slot_bytes=3 << 20) as pool:
        for first in sorted({0, 1, n // 2, n - 1, n, plan["gpu_first"]}):
            r = bench.split_call(pool, paths, sizes, n, pl, exp, first, 3, 4)
            assert r["matched"] == want, first
            assert r["ok"] is False  # the damaged pieces mismatch on whichever side holds them


@pytest.mark.parametrize("pl", [256 * 1024, 1 << 20])
def test_stage_memory_kinds(built, gpu, tmp_path, pl):
    """The pinned stages the readers fill: huge-page mappings registered with
    hipHostRegister (the default) and hipHostMalloc (vx_tuning_stage_huge 0,
    test build), switched back and forth on one context (idle stages are freed
    and reallocated); every verdict equals the pool restatement's, warm and
    with the files evicted (direct reads into the stages)."""
    sys.path.insert(0, ROOT)
    import bench
    from vortex_amd.hash_pool import HashPool

    sizes = [3, 4 * pl + 17, 2 * pl, 0, 3 * pl - 5, pl + 1, 64, 2 * pl + pl // 2]
    paths, exp = _torrent(tmp_path, pl, sizes, 29)
    _damage(paths, pl)
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    with HashPool(pl, slots=3, batch_pieces=4, slot_bytes=3 << 20, hooks=True) as pool:
        for huge in (1, 0, 1):
            pool.lib.vx_tuning_stage_huge(pool._h, huge)
            for cold in (False, True):
                if cold:
                    for p in paths:
                        if os.path.exists(p):
                            bench.drop_cache(p)
                got, _ = pool.verify_files(paths, sizes, pl, exp, io_threads=3)
                assert got == want, (huge, cold)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,backend", [(2, "gloo"), (3, "gloo"), (1, "nccl")])
def test_verify_files_sharded_ranks(built, gpu, tmp_path, world, backend):
    """`world` ranks (all on this box's GPU(s)) each verify their contiguous
    shard; the gathered verdicts equal the one-process oracle.  gloo gathers
    host tensors (several ranks may share the box's one GPU); the nccl case is
    RCCL at world size 1 (RCCL refuses two ranks on one GPU): process-group
    init on the device and the device-tensor all-gather / all-reduce path of
    shard.py, the one the 8-GPU node runs."""
    pl = 256 * 1024
    sizes = [3, 4 * pl + 17, 2 * pl, 0, 3 * pl - 5, pl + 1, 64, 9 * pl + pl // 2]
    paths, exp = _torrent(tmp_path, pl, sizes, 22)
    _damage(paths, pl)
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    spec = tmp_path / "spec.json"
    spec.write_text(json.dumps({"paths": paths, "sizes": sizes, "piece_length": pl, "expected": exp.hex()}))
    out = tmp_path / "out.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "_reverify_rank.py"), str(spec), str(out), backend]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["world"] == world and res["backend"] == backend
    assert res["gather_ok"]
    assert res["matched"] == want
    n = len(want)
    # pieces overlapping the truncated / missing files
    starts = [sum(sizes[:k]) for k in range(len(sizes))]
    lost = set()
    for k, lim in ((4, pl // 3), (5, 0)):
        for i in range(n):
            a, b = i * pl, min((i + 1) * pl, sum(sizes))
            if a < starts[k] + sizes[k] and b > starts[k] + lim:
                lost.add(i)
    assert res["bad"] == len(lost)


@pytest.mark.parametrize("nctx,pl", [(2, 256 * 1024), (3, 1 << 20), (3, 64 * 1024 + 64)])
def test_verify_files_multi_contexts(built, gpu, tmp_path, nctx, pl):
    """vx_verify_files_multi: the in-process multi-device form vortex (one
    process, one event loop) would call — nctx contexts, all on this box's
    device 0 here, each verifying its contiguous range on its own thread.
    Equal to the one-context call and to the oracle, damaged files included;
    the I/O-error count is the same as one context's."""
    from vortex_amd._lib import VX_EINVAL, VxError
    from vortex_amd.hash_pool import HashPool, verify_files_multi

    sizes = [3, 4 * pl + 17, 2 * pl, 0, 3 * pl - 5, pl + 1, 64, 9 * pl + pl // 2]
    paths, exp = _torrent(tmp_path, pl, sizes, 23 + nctx)
    n = len(exp) // 20
    _damage(paths, pl)
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    assert not all(want) and any(want)
    pools = [HashPool(pl, slots=2 + k % 2, slot_bytes=(2 + k) << 20) for k in range(nctx)]
    try:
        one, bad_one = pools[0].verify_files(paths, sizes, pl, exp)
        assert one == want
        for io in (0, 1, 7):
            for p in pools:
                p.reset_stats()
            got, bad = verify_files_multi(pools, paths, sizes, pl, exp, io_threads=io)
            assert got == want and bad == bad_one, io
            # each context counted its own contiguous share (vx_get_stats)
            sts = [p.stats() for p in pools]
            assert sum(st["pieces_completed"] for st in sts) == n
            assert sum(st["io_errors"] for st in sts) == bad
            assert sum(st["bytes_completed"] for st in sts) == sum(sizes)
            assert [st["pieces_completed"] for st in sts] == [n // nctx + (k >= nctx - n % nctx)
                                                               for k in range(nctx)]
        # fewer pieces than contexts: the first contexts get empty ranges
        tiny = tmp_path / "tiny.bin"
        tiny.write_bytes(oracle.gen_piece(5, 5, pl + 1))
        texp = hashlib.sha1(tiny.read_bytes()[:pl]).digest() + bytes(20)  # piece 1 mismatches
        got, bad = verify_files_multi(pools, [str(tiny)], [pl + 1], pl, texp)
        assert got == [True, False] and bad == 0
        with pytest.raises(VxError) as e:
            verify_files_multi([pools[0], pools[0]], paths, sizes, pl, exp)
        assert e.value.code == VX_EINVAL
        with pytest.raises(VxError) as e:  # n_pieces inconsistent with the files
            verify_files_multi(pools, paths, sizes, pl, exp + bytes(20))
        assert e.value.code == VX_EINVAL
    finally:
        for p in pools:
            p.close()


@pytest.mark.parametrize("pl,cold_chunk,direct_io", [(256 * 1024, 0, 1), (2 << 20, 0, 1), (2 << 20, 1 << 20, 1),
                                                     (4 << 20, 1 << 20, 1), (2 << 20, 0, 0), (256 * 1024, 0, 0)])
def test_verify_files_cold_direct_reads(built, gpu, tmp_path, pl, cold_chunk, direct_io):
    """Re-verify of files whose pages are NOT in the page cache: the readers
    take the O_DIRECT path for aligned, uncached ranges (vx_files::DirectIo,
    DESIGN.md §6.1) and the buffered path for the rest (unaligned segments
    where files meet, a short tail).  Verdicts equal the oracle's on the same
    damaged multi-file torrent, and the call's trace shows direct reads when
    the filesystem takes O_DIRECT.  With vx_config.verify_cold_chunk (off by
    default) evicted calls of pieces >= 2 MiB run 1 MiB rounds (many windows
    of the 16 MiB slots); cached ones, and every call by default, 256 KiB.
    With direct_io = 0 every read goes through the page cache (vortex's own
    pread) and the verdicts are the same."""
    import pathlib
    import shutil
    import tempfile

    def takes_direct(d):
        try:
            fd = os.open(os.path.join(d, "probe"), os.O_CREAT | os.O_RDWR | os.O_DIRECT, 0o600)
            os.close(fd)
            return True
        except OSError:
            return False

    # a disk-backed directory when pytest's tmp_path is tmpfs (no O_DIRECT there)
    where, own = tmp_path, None
    if not takes_direct(str(tmp_path)) and os.path.isdir("/var/tmp") and os.access("/var/tmp", os.W_OK):
        own = tempfile.mkdtemp(prefix="vx_cold_", dir="/var/tmp")
        where = pathlib.Path(own)
    direct_ok = takes_direct(str(where))
    print(f"cold re-verify test dir {where}: O_DIRECT {'yes' if direct_ok else 'no'}")
    try:
        _cold_direct_reads(where, pl, cold_chunk, direct_ok, direct_io)
    finally:
        if own:
            shutil.rmtree(own, ignore_errors=True)


def _cold_direct_reads(tmp_path, pl, cold_chunk, direct_ok, direct_io):
    from vortex_amd.hash_pool import HashPool

    sizes = [3 * pl + 4096 * 3, 5 * pl, 2 * pl + 777, pl + 1, 9 * pl]  # aligned and misaligned file starts
    paths, exp = _torrent(tmp_path, pl, sizes, 31)
    with open(paths[1], "r+b") as f:  # one flipped byte in an aligned region
        f.seek(2 * pl + 5000)
        b = f.read(1)
        f.seek(2 * pl + 5000)
        f.write(bytes([b[0] ^ 0x11]))
    want = oracle.pool_verify_files(paths, sizes, pl, exp, threads=4)
    assert not all(want) and any(want)

    def evict():
        for p in paths:
            fd = os.open(p, os.O_RDONLY)
            os.fsync(fd)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            os.close(fd)

    chunked = pl >= 2 << 20
    with HashPool(pl, slots=3, slot_bytes=16 << 20, verify_cold_chunk=cold_chunk, direct_io=direct_io) as pool:
        for _ in range(2):
            evict()
            got, bad = pool.verify_files(paths, sizes, pl, exp, io_threads=4)
            assert got == want and bad == 0
            tr = pool.last_verify()
            assert tr["read_bytes"] == sum(sizes)
            if not direct_io:
                assert tr["direct_bytes"] == 0
                assert tr["chunk_bytes"] == (256 * 1024 if chunked else 0), tr
            elif direct_ok:
                assert tr["direct_bytes"] > 0
                assert tr["chunk_bytes"] == ((cold_chunk or 256 * 1024) if chunked else 0), tr
        # half cached: each file's first half in the page cache, the second not -> the
        # file is probed per read; the uncached aligned ranges go direct, verdicts unchanged
        evict()
        for p in paths:
            fd = os.open(p, os.O_RDONLY)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_RANDOM)  # no readahead past the half
            size = os.fstat(fd).st_size
            os.pread(fd, size // 2, 0)
            os.close(fd)
        got, bad = pool.verify_files(paths, sizes, pl, exp, io_threads=4)
        tr = pool.last_verify()
        assert got == want and bad == 0
        if direct_io and direct_ok:
            assert 0 < tr["direct_bytes"] < sum(sizes), tr
        # cached now (the buffered reads above filled part of it; read the rest): no direct reads
        for p in paths:
            with open(p, "rb") as f:
                while f.read(1 << 20):
                    pass
        got, bad = pool.verify_files(paths, sizes, pl, exp, io_threads=4)
        tr = pool.last_verify()
        assert got == want and tr["direct_bytes"] == 0
        assert tr["chunk_bytes"] == (256 * 1024 if chunked else 0), tr
