"""Two ranks on one GPU over gloo: do all_gather_into_tensor / all_to_all_single take CUDA
tensors? (decides whether the replica group can be exercised end to end on a 1-GPU box)"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def run(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = torch.full((8,), rank, dtype=torch.uint8, device="cuda:0")
    out = torch.empty(8 * world, dtype=torch.uint8, device="cuda:0")
    try:
        dist.all_gather_into_tensor(out, x)
        print(rank, "all_gather_into_tensor ok", out.tolist(), flush=True)
    except Exception as e:
        print(rank, "all_gather_into_tensor FAIL", repr(e)[:200], flush=True)
    y = torch.arange(8, dtype=torch.int32, device="cuda:0") + 100 * rank
    o = torch.empty_like(y)
    try:
        dist.all_to_all_single(o, y)
        print(rank, "all_to_all_single ok", o.tolist(), flush=True)
    except Exception as e:
        print(rank, "all_to_all_single FAIL", repr(e)[:200], flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(run, args=(2, int(sys.argv[1]) if len(sys.argv) > 1 else 29533), nprocs=2)
