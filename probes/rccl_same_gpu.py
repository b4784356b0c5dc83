"""Diagnostics (not product, not tests): can two ranks on the box's one GPU
talk over RCCL (the `nccl` backend)?  If so, the gather's nccl branch
(distributed.gather_packed / ChunkSender / ChunkReceiver) runs here.
usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
       --master-port 29531 probes/rccl_same_gpu.py"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    x = torch.full((4,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    print(f"rank {rank}: all_reduce {x.tolist()}", flush=True)
    from scanner_colmap_amd.distributed import ChunkReceiver, ChunkSender, gather_packed
    rng = np.random.default_rng(rank)
    offs = np.array([0, 5, 9], dtype=np.int64)
    data = rng.integers(0, 255, 9, dtype=np.uint8)
    g = gather_packed(offs, data, dev)
    if rank == 0:
        ok = all(np.array_equal(g[r][1], np.random.default_rng(r).integers(0, 255, 9, dtype=np.uint8))
                 for r in range(world))
        print(f"gather_packed over nccl: {'equal' if ok else 'DIFFERENT'}", flush=True)

    class P:
        def __init__(self, o, d):
            self.offsets, self.data = o, d
    chunks = [(np.array([0, 3], np.int64), rng.integers(0, 255, 3, dtype=np.uint8)) for _ in range(3)]
    if rank == 0:
        recv = ChunkReceiver(world, dev)
        per = recv.result()
        print(f"chunks from rank 1: {len(per[1])}", flush=True)
    else:
        snd = ChunkSender(dev)
        for o, d in chunks:
            snd.submit(P(o, d))
        snd.finish()
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank}: done", flush=True)


if __name__ == "__main__":
    main()
