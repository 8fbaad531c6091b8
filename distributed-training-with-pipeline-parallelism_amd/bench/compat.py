"""Reference-compatible benchmark API (reference helper:98-235, notebook cells 19-26).

* :func:`run_train_iterations` -- 2 untimed warmup steps, ``num_iterations`` timed
  ``schedule.step`` calls; returns ``{'elapsed_time','throughput','tokens_processed'}``
  (helper:98-143).  Timing matches the reference (wall clock on the calling rank,
  global tokens), with a device synchronize so GPU work is inside the window.
* :func:`worker_process` -- per-rank bootstrap (helper:150-235): rendezvous, group
  init (gloo on CPU, RCCL on GPU), the interleave rule (v=2 iff
  ``n_layers % (2*world) == 0``, helper:181-185), synthetic tokens, token-wise CE
  loss, loop placement ``stage = rank + world*i`` (helper:204-211), schedule factory
  with ``num_mb`` microbatches (default 4, helper:214), last-rank result reporting
  and ``{'error': ...}`` capture (helper:226-235).
* :func:`run_one_experiment`, :func:`run_all_experiments`,
  :func:`compute_speedup_and_efficiency` -- the notebook's launcher, sweep and
  analysis (nb:306-333, nb:345-392, nb:405-433), with a per-experiment timeout and a
  free port per run instead of the reference's fixed 29500 + unbounded join
  (SURVEY §2.8 item 11).

``engine='native'`` (the default whenever a GPU is present) runs the same reference
architecture on the MI355X HIP path (explicit backward, hand-written kernels) at the
reference's own precision (``precision='fp32'``: the f32 MFMA GEMM / f32 flash attention /
f32 norm, CE and embedding kernels; ``'bf16'`` is the fast path), with per-microbatch HIP
graphs, the native step tape and -- one process -- microbatch lanes; its last rank's
``step()`` returns the merged ``[B, S, vocab]`` logits like the reference's (persistent
graph outputs, so the tape replays that step too).  ``engine='torch'`` is the nn.Module /
autograd path the reference uses (the CPU default).  Every metrics dict also carries the
measured and analytic pipeline bubble, the precision and the execution path.
"""
from __future__ import annotations

import os
import socket
import time
import traceback
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..models.ref_transformer import ModelArgs, Transformer, manual_model_split, tokenwise_loss_fn
from ..parallel.api import get_schedule_class


def _sync(device) -> None:
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize()


def run_train_iterations(schedule, x: torch.Tensor, y: torch.Tensor, rank: int, world_size: int,
                         num_iterations: int = 10, warmup: int = 2, device=None,
                         measure_bubble: bool = True) -> Dict[str, float]:
    """Reference timed loop (helper:98-143) + one extra profiled step (untimed) for the
    measured pipeline bubble ``1 - sum(busy_r) / (P * max step_r)`` over the schedule's
    group, reported with the analytic (P-1)/(v*m+P-1) of the same schedule."""
    total_toks = x.shape[0] * x.shape[1] * num_iterations
    first = rank == 0
    last = rank == world_size - 1
    dev = device if device is not None else x.device

    def one():
        if first and last:
            schedule.step(x, target=y, losses=[])
        elif first:
            schedule.step(x)
        elif last:
            schedule.step(target=y, losses=[])
        else:
            schedule.step()

    for _ in range(warmup):
        one()
    _sync(dev)
    start_t = time.time()
    for _ in range(num_iterations):
        one()
    _sync(dev)
    elapsed = time.time() - start_t
    out = {"elapsed_time": elapsed, "throughput": total_toks / elapsed, "tokens_processed": total_toks}
    rt = getattr(schedule, "runtime", None)
    if rt is not None:
        st0 = next(iter(rt.stages.values()))
        arena = getattr(st0, "arena", None)
        if arena is not None:
            out["precision"] = "fp32" if arena.dtype == torch.float32 else "bf16"
        else:   # (a stage the reference's split left without layers has no parameters)
            p0 = next(iter(st0.submod.parameters()), None)
            out["precision"] = str(p0.dtype).replace("torch.", "") if p0 is not None else str(x.dtype)
        out["native_runner"] = rt.native_runner is not None
        out["native_reason"] = rt.native_reason
        out["lanes"] = rt.lanes
    if measure_bubble and rt is not None:
        from ..parallel.schedules import analytic_bubble
        if dist.is_initialized() and world_size > 1:
            dist.barrier()
        rt.profile = True
        try:
            one()
        finally:
            rt.profile = False
        mine = torch.tensor([rt.busy_ms(), rt.last_step_ms], dtype=torch.float64)
        if dist.is_initialized() and world_size > 1:
            t = mine.to(dev) if dist.get_backend() == "nccl" else mine
            allv = [torch.zeros_like(t) for _ in range(world_size)]
            dist.all_gather(allv, t)
            allv = [v.cpu() for v in allv]
        else:
            allv = [mine]
        step = max(float(v[1]) for v in allv)
        out["bubble_fraction"] = (1.0 - sum(float(v[0]) for v in allv) / (len(allv) * step)) if step > 0 else None
        out["analytic_bubble"] = analytic_bubble(rt.schedule, rt.pp, rt.m, rt.v)
    return out


def stages_per_worker(schedule_type: str, n_layers: int, world_size: int) -> int:
    """Interleave policy (helper:181-183)."""
    return 2 if schedule_type == "Interleaved1F1B" and n_layers % (world_size * 2) == 0 else 1


def native_reference_schedule(args: ModelArgs, schedule_type: str, rank: int, world_size: int, batch_size: int,
                              seq_length: int, num_microbatches: int, device, precision: str = "fp32",
                              lanes: Optional[int] = None, p2p=None):
    """The reference's per-rank setup (helper:180-220: interleave rule, loop placement
    ``stage = rank + world*i``, schedule factory) on the native path: build_reference_stage
    per local stage (f32 or bf16 kernels, HIP graphs on GPUs), the schedule class, and --
    with one process on a GPU -- microbatch lanes as PipelineTrainer picks them."""
    from ..models.stage import build_reference_stage
    dev = torch.device(device)
    spw = stages_per_worker(schedule_type, args.n_layers, world_size)
    num_stages = world_size * spw
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[precision]
    stages = [build_reference_stage(args, rank + world_size * i, num_stages, dev, dtype=dt,
                                    mbs=batch_size // num_microbatches, seq_len=seq_length) for i in range(spw)]
    cls = get_schedule_class(schedule_type)
    schedule = cls(stages if spw > 1 or schedule_type == "Interleaved1F1B" else stages[0],
                   n_microbatches=num_microbatches, loss_fn=tokenwise_loss_fn(args.vocab_size), p2p=p2p)
    if dev.type == "cuda":
        from ..engine import auto_lanes
        st = stages[0]
        n = lanes if lanes is not None else auto_lanes(
            st.cfg, world_size, spw, True, dev, num_microbatches, st.mbs * st.S, st.arena.numel,
            st.model.layer_range[1] - st.model.layer_range[0])
        schedule.runtime.set_lanes(n)
    return schedule


def worker_process(rank, world_size, n_layers, n_heads, schedule_type, batch_size, seq_length, num_iterations,
                   results_queue, num_microbatches: int = 4, device: Optional[str] = None, port: int = 29500,
                   engine: str = "auto", dropout: float = 0.1, seed: Optional[int] = None, precision: str = "fp32",
                   lanes: Optional[int] = None):
    """Reference worker (helper:150-235).  ``engine='auto'`` (default): the MI355X HIP path
    (``native``: hand-written kernels, explicit backward) when a GPU is present, the
    reference's nn.Module / autograd path (``torch``) on CPU.  ``MIPIPE_DIST_BACKEND=gloo``
    with GPUs: ranks share the visible devices and gloo carries the traffic (a test mode
    for one-GPU boxes)."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        os.environ["RANK"] = str(rank)
        os.environ["LOCAL_RANK"] = str(rank)
        os.environ["WORLD_SIZE"] = str(world_size)
        use_gpu = (device == "cuda") or (device is None and torch.cuda.is_available())
        if engine == "auto":
            engine = "native" if use_gpu else "torch"
        if use_gpu and os.environ.get("MIPIPE_DIST_BACKEND") == "gloo":
            dev = torch.device("cuda", rank % torch.cuda.device_count())
            torch.cuda.set_device(dev)
            dist.init_process_group(backend="gloo", rank=rank, world_size=world_size)
        elif use_gpu:
            torch.cuda.set_device(rank)
            dev = torch.device("cuda", rank)
            dist.init_process_group(backend="nccl", rank=rank, world_size=world_size, device_id=dev)
        else:
            dev = torch.device("cpu")
            dist.init_process_group(backend="gloo", rank=rank, world_size=world_size)
        if seed is not None:
            torch.manual_seed(seed)
        spw = stages_per_worker(schedule_type, n_layers, world_size)
        num_stages = world_size * spw
        args = ModelArgs(n_layers=n_layers, n_heads=n_heads, dropout=dropout)
        x = torch.randint(0, args.vocab_size, (batch_size, seq_length), dtype=torch.long, device=dev)
        y = torch.randint(0, args.vocab_size, (batch_size, seq_length), dtype=torch.long, device=dev)
        if engine == "native":
            schedule = native_reference_schedule(args, schedule_type, rank, world_size, batch_size, seq_length,
                                                 num_microbatches, dev, precision=precision, lanes=lanes)
        else:
            stages = []
            for i in range(spw):
                model = Transformer(args)
                st = manual_model_split(model, rank + world_size * i, num_stages, dev)
                st.graphs = use_gpu   # the user module's fwd/bwd replayed as HIP graphs per microbatch slot
                stages.append(st)
            cls = get_schedule_class(schedule_type)
            schedule = cls(stages if spw > 1 or schedule_type == "Interleaved1F1B" else stages[0],
                           n_microbatches=num_microbatches, loss_fn=tokenwise_loss_fn(args.vocab_size))
        metrics = run_train_iterations(schedule, x, y, rank, world_size, num_iterations, device=dev)
        if rank == world_size - 1:
            results_queue.put(metrics)
        dist.destroy_process_group()
    except Exception as e:  # reference helper:231-235
        print(f"Error in rank {rank}: {e}")
        traceback.print_exc()
        results_queue.put({"error": str(e)})


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_one_experiment(n_layers, n_heads, num_processes, schedule_type, batch_size=32, seq_length=128,
                       num_iterations=10, timeout: float = 900.0, **kw) -> Dict:
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker_process, args=(r, num_processes, n_layers, n_heads, schedule_type, batch_size,
                                                        seq_length, num_iterations, q), kwargs=dict(port=port, **kw))
             for r in range(num_processes)]
    for p in procs:
        p.start()
    deadline = time.time() + timeout
    result = None
    try:
        result = q.get(timeout=timeout)
    except Exception:
        result = {"error": "No results returned"}
    for p in procs:
        p.join(timeout=max(1.0, deadline - time.time()))
        if p.is_alive():
            p.terminate()
            p.join(5)
    return result


def run_all_experiments(n_heads_list=(4, 8, 12), n_layers_list=(4, 8, 12), num_processes_list=(2, 4),
                        schedules=("GPipe", "1F1B", "Interleaved1F1B"), num_iterations=5, **kw):
    import pandas as pd
    rows = []
    for n_heads in n_heads_list:
        for n_layers in n_layers_list:
            for P in num_processes_list:
                for sched in schedules:
                    try:
                        m = run_one_experiment(n_layers, n_heads, P, sched, num_iterations=num_iterations, **kw)
                        if "error" not in m:
                            rows.append(dict(n_layers=n_layers, n_heads=n_heads, num_processes=P, schedule=sched,
                                             throughput=m["throughput"], elapsed_time=m["elapsed_time"],
                                             tokens_processed=m["tokens_processed"],
                                             bubble_fraction=m.get("bubble_fraction"),
                                             analytic_bubble=m.get("analytic_bubble")))
                            print(f"L{n_layers} H{n_heads} P{P} {sched}: {m['throughput']:.1f} tok/s")
                        else:
                            print(f"L{n_layers} H{n_heads} P{P} {sched}: error {m['error']}")
                    except Exception as e:  # nb:388-390
                        print(f"experiment failed: {e}")
    return pd.DataFrame(rows)


def compute_speedup_and_efficiency(df):
    """speedup = thr / thr_GPipe for the same (L,H,P); efficiency = speedup / P * 100 (nb:403-433)."""
    import pandas as pd
    out = []
    for (L, H, P), g in df.groupby(["n_layers", "n_heads", "num_processes"]):
        base = g[g["schedule"] == "GPipe"]["throughput"]
        if base.empty:
            continue
        b = float(base.iloc[0])
        for _, row in g.iterrows():
            if row["schedule"] == "GPipe":
                continue
            sp = row["throughput"] / b
            out.append(dict(n_layers=L, n_heads=H, num_processes=P, schedule=row["schedule"],
                            throughput=row["throughput"], speedup=sp, efficiency=sp / P * 100))
    return pd.DataFrame(out)


def throughput_pivot(df):
    """Mean throughput by (layers, heads) x (schedule, processes) -- the notebook's
    summary table (nb:766-782)."""
    return df.pivot_table(index=["n_layers", "n_heads"], columns=["schedule", "num_processes"], values="throughput",
                          aggfunc="mean")


def plot_speedup_efficiency(eff_df, path: str) -> None:
    """1x2 figure: speedup vs GPipe and 'efficiency' per L{L}_H{H} config (nb:880-941)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig, axes = plt.subplots(1, 2, figsize=(14, 5))
    for (sched, P), g in eff_df.groupby(["schedule", "num_processes"]):
        labels = [f"L{l}_H{h}" for l, h in zip(g["n_layers"], g["n_heads"])]
        axes[0].plot(labels, g["speedup"], marker="o", label=f"{sched} P={P}")
        axes[1].plot(labels, g["efficiency"], marker="o", label=f"{sched} P={P}")
    axes[0].set_title("speedup vs GPipe")
    axes[1].set_title("efficiency = speedup / P x 100")
    for ax in axes:
        ax.tick_params(axis="x", rotation=45)
        ax.legend(fontsize=8)
    fig.tight_layout()
    fig.savefig(path)
    plt.close(fig)


def plot_throughput(df, path: str) -> None:
    """Grid of throughput vs processes per (L, H), one line per schedule (nb:972-1002)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    Ls, Hs = sorted(df["n_layers"].unique()), sorted(df["n_heads"].unique())
    fig, axes = plt.subplots(len(Ls), len(Hs), figsize=(4 * len(Hs), 3 * len(Ls)), squeeze=False)
    for i, L in enumerate(Ls):
        for j, H in enumerate(Hs):
            ax = axes[i][j]
            g = df[(df["n_layers"] == L) & (df["n_heads"] == H)]
            for sched, gs in g.groupby("schedule"):
                gs = gs.sort_values("num_processes")
                ax.plot(gs["num_processes"], gs["throughput"], marker="o", label=sched)
            ax.set_title(f"L={L} H={H}")
            ax.set_xlabel("processes")
            ax.set_ylabel("tok/s")
            ax.legend(fontsize=7)
    fig.tight_layout()
    fig.savefig(path)
    plt.close(fig)


def environment_report() -> dict:
    """Torch / ROCm / device report (the notebook's environment cell, nb:256-259)."""
    import os as _os
    rep = {"torch": torch.__version__, "hip": getattr(torch.version, "hip", None),
           "gpu_available": torch.cuda.is_available(), "cpu_count": _os.cpu_count()}
    if torch.cuda.is_available():
        rep["devices"] = [torch.cuda.get_device_name(i) for i in range(torch.cuda.device_count())]
    for k, v in rep.items():
        print(f"{k}: {v}")
    return rep
