"""Spawn a CPU/gloo process group of `world` ranks running `fn(rank, world, *args)`."""
import os
import socket
import sys
import traceback

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, q):
    try:
        if ROOT not in sys.path:
            sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                          WORLD_SIZE=str(world))
        import torch
        import torch.distributed as dist
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        out = fn(rank, world, *args)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok", out))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


def run_world(fn, world, *args, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in ps:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, status, out = q.get(timeout=timeout)
            if status != "ok":
                raise RuntimeError(f"rank {rank} failed:\n{out}")
            results[rank] = out
    finally:
        for p in ps:
            p.join(10)
            if p.is_alive():
                p.terminate()
    return results
