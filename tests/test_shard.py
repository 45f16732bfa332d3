"""CPU: the multi-GPU shard plan and the verdict gather, on gloo with
world_size 2 and 3 (the same code runs over RCCL on the GPU node)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vortex_amd.shard import blocks, gather_verdicts, shard_range, shard_ragged


def test_shard_range_covers_exactly():
    for n in (0, 1, 7, 65536, 524288, 1387):
        for w in (1, 2, 3, 4, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            pos = 0
            for s, c in spans:
                assert s == pos
                pos += c
            assert pos == n
            counts = [c for _, c in spans]
            assert max(counts) - min(counts) <= 1
            assert counts == sorted(counts)  # remainder goes to the last ranks
    assert shard_range(524288, 8, 3) == (3 * 65536, 65536)


def test_shard_ragged_balances_blocks():
    lens = [4 << 20] * 4 + [1 << 20] * 16 + [16384] * 1024
    plan = shard_ragged(lens, 4)
    assert sorted(i for p in plan for i in p) == list(range(len(lens)))
    loads = [sum(blocks(lens[i]) for i in p) for p in plan]
    assert max(loads) - min(loads) <= blocks(4 << 20)
    for p in plan:
        assert [lens[i] for i in p] == sorted((lens[i] for i in p), reverse=True)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, count = shard_range(n_total, world, rank)
        # "verdict" of global piece g is (g % 5 != 0)
        local = torch.tensor([(g % 5 != 0) for g in range(start, start + count)], dtype=torch.uint8)
        full = gather_verdicts(local, n_total)
        q.put((rank, full.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total", [(2, 1001), (3, 65536 + 2)])
def test_gather_verdicts_gloo(world, n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [int(g % 5 != 0) for g in range(n_total)]
    for r in range(world):
        assert results[r] == want


class _OraclePool:
    """Stands in for HashPool on CPU: verify_files over a piece range, with
    the oracle's restatement of the bulk re-verify as the verdict source."""

    def verify_files(self, paths, lens, pl, expected, io_threads=0, first=0, count=None):
        import oracle

        full = oracle.pool_verify_files(paths, lens, pl, expected, threads=2)
        count = len(full) - first if count is None else count
        self.seen = (first, count)
        return full[first:first + count], 0


def _reverify_worker(rank, world, port, spec, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vortex_amd.shard import verify_files_sharded

        pool = _OraclePool()
        got, bad = verify_files_sharded(pool, *spec)
        q.put((rank, got, bad, pool.seen))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_verify_files_sharded_gloo(tmp_path, world):
    """Each rank asks for exactly its shard_range and every rank gets the whole
    torrent's verdicts back in piece order."""
    import hashlib

    import oracle

    pl = 16384
    sizes = [100, 5 * pl + 3, 0, 2 * pl]
    paths = []
    for k, L in enumerate(sizes):
        p = tmp_path / f"f{k}"
        p.write_bytes(oracle.gen_piece(3, k, L))
        paths.append(str(p))
    data = b"".join(open(p, "rb").read() for p in paths)
    exp = bytearray(b"".join(hashlib.sha1(data[i:i + pl]).digest() for i in range(0, len(data), pl)))
    exp[20 * 2] ^= 1  # piece 2 mismatches
    n = len(exp) // 20
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    spec = (paths, sizes, pl, bytes(exp))
    procs = [ctx.Process(target=_reverify_worker, args=(r, world, port, spec, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (g, b, s) for r, g, b, s in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [i != 2 for i in range(n)]
    for r in range(world):
        assert res[r][0] == want and res[r][1] == 0
        assert res[r][2] == shard_range(n, world, r)
