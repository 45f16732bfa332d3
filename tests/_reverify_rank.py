"""One rank of the multi-GPU re-verify test (tests/test_gpu_reverify_shard.py).

Launched by torch.distributed.run; every rank opens a HashPool on its GPU
(LOCAL_RANK modulo the visible devices, so two ranks share cuda:0 on a
one-GPU box), verifies its shard with vx_verify_files_range and gathers the
verdicts (shard.verify_files_sharded).  Rank 0 writes the result as JSON.
"""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vortex_amd import shard  # noqa: E402
from vortex_amd.hash_pool import HashPool  # noqa: E402


def main():
    spec = json.load(open(sys.argv[1]))
    backend = sys.argv[3] if len(sys.argv) > 3 else "gloo"
    dev = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    if backend == "nccl":  # RCCL: device tensors, one GPU per rank
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group(backend)
    with HashPool(spec["piece_length"], device=dev, slots=3, batch_pieces=8, slot_bytes=4 << 20) as pool:
        got, bad = shard.verify_files_sharded(pool, spec["paths"], spec["sizes"], spec["piece_length"],
                                              bytes.fromhex(spec["expected"]), io_threads=3)
    # the verdict gather on its own, from a device tensor: RCCL gathers it in place on the GPU
    world, rank = dist.get_world_size(), dist.get_rank()
    n_total = 1001
    start, count = shard.shard_range(n_total, world, rank)
    local = torch.tensor([(g % 7 != 0) for g in range(start, start + count)], dtype=torch.uint8, device="cuda")
    full = shard.gather_verdicts(local, n_total)
    gather_ok = full.device == local.device and full.cpu().tolist() == [int(g % 7 != 0) for g in range(n_total)]
    if rank == 0:
        with open(sys.argv[2], "w") as f:
            json.dump({"matched": got, "bad": bad, "world": world, "backend": dist.get_backend(),
                       "gather_ok": gather_ok}, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
