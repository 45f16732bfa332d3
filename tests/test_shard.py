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
