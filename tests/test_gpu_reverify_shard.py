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


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_verify_files_sharded_ranks(built, gpu, tmp_path, world):
    """`world` ranks (all on this box's GPU(s), gloo for the gather) each verify
    their contiguous shard; the gathered verdicts equal the one-process oracle."""
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
           os.path.join(ROOT, "tests", "_reverify_rank.py"), str(spec), str(out), "gloo"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["world"] == world
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
