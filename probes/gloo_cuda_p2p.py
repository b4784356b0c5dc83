"""Diagnostics (not product, not tests): does gloo send/recv device tensors?
If so, the gather's device-staging branch (distributed.py, on_gpu) can run
with two ranks on the box's one GPU.
usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
       --master-port 29533 probes/gloo_cuda_p2p.py"""
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
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.full((8,), rank + 1, dtype=torch.uint8, device=dev)
    try:
        if rank == 1:
            for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, t, 0)]):
                w.wait()
        else:
            r = torch.empty(8, dtype=torch.uint8, device=dev)
            for w in dist.batch_isend_irecv([dist.P2POp(dist.irecv, r, 1)]):
                w.wait()
            print(f"gloo device p2p: {r.cpu().tolist()}", flush=True)
    except Exception as e:  # report, do not hang the peer
        print(f"rank {rank}: gloo device p2p refused: {e}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
