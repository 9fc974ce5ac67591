"""Probe: can two RCCL ranks share the one GPU of a gpurun box? (all_reduce + gather of device
uint8 buffers, the two collectives fastvideocodec_amd.dist uses). Prints one line per rank."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    t = torch.tensor([float(rank + 1)], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    buf = torch.full((1000,), rank + 7, dtype=torch.uint8, device=dev)
    outs = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, outs, dst=0)
    torch.cuda.synchronize()
    ok = float(t.item()) == float(world) and (rank != 0 or all(int(o[0]) == r + 7 for r, o in enumerate(outs)))
    print(f"rank {rank}: all_reduce max {t.item()} gather ok {ok}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mp.start_processes(worker, args=(world, 29533), nprocs=world, start_method="spawn")
