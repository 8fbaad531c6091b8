"""Can two RCCL ranks share one GPU on this image?  2 processes on cuda:0, nccl backend,
one all_reduce and one send/recv; prints what happened (used to decide whether multi-rank
RCCL tests can run on a one-GPU box)."""
import os
import sys
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def work(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=2, device_id=torch.device("cuda", 0))
    t = torch.full((4,), float(rank + 1), device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    x = torch.arange(8, device="cuda", dtype=torch.float32)
    if rank == 0:
        dist.send(x, 1)
    else:
        y = torch.zeros(8, device="cuda")
        dist.recv(y, 0)
        torch.cuda.synchronize()
        print("rank1 recv ok", bool((y == x).all()), flush=True)
    print(f"rank {rank} all_reduce -> {t.tolist()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    port = int(sys.argv[1]) if len(sys.argv) > 1 else 29611
    mp.start_processes(work, args=(port,), nprocs=2, start_method="spawn")
