#!/usr/bin/env python3
"""Flagship benchmark: GPT-2 pipeline-parallel training throughput on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model gpt2-small]
                    [--schedule 1F1B] [--mbs MBS] [--seq 1024] [--microbatches M]

N GPUs = N pipeline stages (PP=N, one process per GPU); for N>1 the driver launches it
with torch.distributed.run (if launched without it, this script re-launches itself under
torch.distributed.run).  Work per GPU is fixed as N grows ("weak" scaling): every GPU
runs 128 sequences of ``seq`` tokens through all of its layers per step, so the global
batch is 128 N sequences.  A pipeline (N > 1) splits it into ``microbatches = 4*N`` of
``mbs = 32`` sequences: m = 4P rather than 2P takes the 1F1B bubble (P-1)/(m+P-1) at P = 8
from 0.30 to 0.18 (planned efficiency of the lowered program with the distributed head
0.72 -> 0.83, tools/schedule_table.py); at P = 8 the global batch is 1M tokens.  One GPU
has no bubble to amortise and runs 2 microbatches of 64 (the two microbatch lanes overlap
them): 990.5K / 991.8K tok/s vs 978.6K / 978.3K as 4 x 32 (profiles/r3_bench_mbs64_ab.txt;
one stream: 64 -> 978K, 32 -> 929K, 16 -> 880K, profiles/r3_lane1_mbs_ab.txt).  Each timed step is a full training step: all
microbatch forwards/backwards through the lowered schedule, p2p of activations and
gradients, grad-norm clip and the fused AdamW update.

Execution path (the same at every N): per-microbatch stage compute replayed as HIP graphs,
one step recorded as a native instruction tape (csrc/runtime/stage_runner.cpp) and replayed
from C++; p2p on the native RCCL engine (one communicator + stream per direction,
csrc/comm/rccl_p2p.h), pre-flight pinged at init with an in-process fallback to torch p2p.
The JSON reports which path ran (``hip_graphs``, ``native_runner``, ``p2p``).

Hang safety (N>1): the pipeline program is PROVEN hang-free before it runs
(PipelineRuntime._prove: every collective after the step's p2p, serial queue model), and
every rank runs the benchmark in a child process under a supervisor.  The child arms a
watchdog over init, warmup, every timed step and the bubble step (on a stall it prints the
program grid + all stacks and exits non-zero); the process-group timeout is 300 s.  If an
attempt fails on any rank, all supervisors retry in a more conservative mode (torch p2p,
then no HIP graphs) on a fresh rendezvous port; the ``attempt`` field says which one
produced the number.  One global deadline (MIPIPE_BENCH_DEADLINE_S, default 540 s, under
the driver's 600 s) bounds all attempts together: each gets at most what is left of it
(and at most MIPIPE_BENCH_ATTEMPT_S, default 240 s), its watchdogs are clamped to that,
and no attempt starts with less than 30 s left.  Supervisors never touch the GPU.

The measured bubble comes from one extra profiled step replayed from the same native tape
(timing events around every graph on the compute stream): ``1 - sum(busy_r) / (P * step)``
with ``step`` the slowest rank's step time, next to the analytic (P-1)/(v*m+P-1).

Prints ONE JSON line on rank 0 (value = whole-job tokens/s, max elapsed over ranks).
Random-init weights, synthetic uniform tokens (no dataset / checkpoint access).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = ("tokens/sec/node + pipeline bubble fraction, GPT-2 PP=1/2/4/8 (GPipe vs 1F1B vs interleaved)")
# The reference publishes only its fp32 toy model on a 10-core CPU; there is
# no same-model/same-precision number to divide by, so vs_baseline is null (see
# tools/ref_table_gpu.py for the reference's own configs run on this framework).
BASELINE_NOTE = ("no same-config reference number: BASELINE.md only has the reference's fp32 toy model "
                 "(L4-12, d768, seq 128) on a 10-core CPU/gloo; see profiles/ for that table on MI355X")

# supervisor attempts: (p2p transport, HIP graphs + native tape)
ATTEMPTS = [("auto", 1), ("torch", 1), ("torch", 0)]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--schedule", default="1F1B")
    ap.add_argument("--mbs", type=int, default=None,
                    help="sequences per microbatch (default: 64 on one GPU, 32 with a pipeline)")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--microbatches", type=int, default=None)
    ap.add_argument("--dp", type=int, default=1)
    # (not "--v": torch.distributed.run's argparse would take it for an abbreviation of
    # its --virtual-local-rank even after the script name)
    ap.add_argument("--vstages", type=int, default=None, help="virtual stages per rank (interleaved)")
    ap.add_argument("--recompute", nargs="?", const="1", default="0", choices=["0", "1", "auto"],
                    help="activation recompute: 1 (on), 0 (off), auto (HBM plan: only if the stash does not fit)")
    ap.add_argument("--graphs", type=int, default=None,
                    help="replay per-microbatch stage compute as HIP graphs + native tape (default: on with a GPU)")
    ap.add_argument("--no-split-head", action="store_true",
                    help="keep the LM head on the last stage (default with PP>1: distributed head)")
    ap.add_argument("--no-bubble", action="store_true", help="skip the profiled bubble-measurement step")
    ap.add_argument("--trace", default=None, help="write a Chrome trace of the profiled step (per rank)")
    ap.add_argument("--step-timeout", type=float, default=None,
                    help="watchdog limit per timed step in s (default 60; 180 for init and the first steps)")
    ap.add_argument("--max-attempts", type=int, default=len(ATTEMPTS), help="supervisor attempts (N>1)")
    ap.add_argument("--no-supervise", action="store_true", help="N>1: run in this process (no retry)")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32"], help="default bf16 on GPU, fp32 on CPU")
    ap.add_argument("--vocab", type=int, default=None, help="override the vocabulary (CPU tests)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------ supervisor
def _attempt_dir() -> str:
    # one node (--nnodes=1): every rank's supervisor is a child of the same launcher agent
    d = os.path.join(os.environ.get("TMPDIR", "/tmp"),
                     f"mipipe_bench_{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}")
    os.makedirs(d, exist_ok=True)
    return d


def _wait_file(path: str, timeout_s: float):
    t_end = time.monotonic() + timeout_s
    while time.monotonic() < t_end:
        if os.path.exists(path):
            with open(path) as f:
                return f.read().strip()
        time.sleep(0.2)
    return None


DEADLINE_S = 540.0       # all attempts together (the driver kills the bench at 600 s)
ATTEMPT_CAP_S = 240.0    # one attempt at most
MIN_ATTEMPT_S = 30.0     # no attempt starts with less than this left


def attempt_budget(elapsed: float, deadline: float = DEADLINE_S, cap: float = ATTEMPT_CAP_S) -> float:
    """Seconds the next attempt may run (0: none may start) -- what is left of the global
    deadline, less a 5 s margin for killing a child, capped per attempt."""
    left = deadline - elapsed - 5.0
    return 0.0 if left < MIN_ATTEMPT_S else min(cap, left)


def supervise(a, argv) -> int:
    """Run the benchmark in a child process per attempt (module docstring).  Rank 0 decides
    after each attempt (did its child print the JSON line?  is there time for another?)
    and publishes the verdict (done | retry | giveup) in a per-launch directory; the other
    ranks follow it.  Never initialises the GPU."""
    t_start = time.monotonic()
    rank = int(os.environ.get("RANK", "0"))
    base_port = int(os.environ.get("MASTER_PORT", "29500"))
    d = _attempt_dir()
    attempts = ATTEMPTS[: max(1, a.max_attempts)]
    if a.graphs is not None or os.environ.get("MIPIPE_P2P"):
        attempts = [(os.environ.get("MIPIPE_P2P", "auto"), 1 if a.graphs is None else a.graphs)] + attempts[1:]
    deadline = float(os.environ.get("MIPIPE_BENCH_DEADLINE_S", str(DEADLINE_S)))
    cap = float(os.environ.get("MIPIPE_BENCH_ATTEMPT_S", str(ATTEMPT_CAP_S)))
    current = {"proc": None}

    def on_term(signum, frame):   # the launcher tears the job down: take the child with us
        p = current["proc"]
        if p is not None and p.poll() is None:
            p.kill()
        os._exit(128 + signum)
    import signal
    signal.signal(signal.SIGTERM, on_term)
    signal.signal(signal.SIGINT, on_term)
    for k, (p2p, graphs) in enumerate(attempts):
        per_attempt_s = attempt_budget(time.monotonic() - t_start, deadline, cap)
        if per_attempt_s <= 0:      # (rank 0 published "giveup" for the previous attempt)
            break
        env = dict(os.environ, MIPIPE_BENCH_CHILD="1", MIPIPE_P2P=p2p, MIPIPE_BENCH_ATTEMPT=str(k),
                   MASTER_PORT=str(base_port + 1 + k), MIPIPE_BENCH_ATTEMPT_S=f"{per_attempt_s:.0f}")
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)   # fresh rendezvous store per attempt
        cmd = [sys.executable, os.path.abspath(__file__)] + list(argv) + ["--graphs", str(graphs)]
        printed = False
        proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if rank == 0 else None, text=True)
        current["proc"] = proc
        t_end = time.monotonic() + per_attempt_s
        if rank == 0:
            import threading

            def pump():
                nonlocal printed
                for line in proc.stdout:
                    if line.lstrip().startswith("{") and '"metric"' in line:
                        printed = True
                    sys.stdout.write(line)
                    sys.stdout.flush()
            th = threading.Thread(target=pump, daemon=True)
            th.start()
        # wait for the child; once the result is in (rank 0 printed it / published "done"),
        # a child still tearing down gets a grace period, then is killed
        vpath = os.path.join(d, f"attempt{k}.verdict")
        done_at = None
        while proc.poll() is None:
            now = time.monotonic()
            if done_at is None and (printed if rank == 0 else os.path.exists(vpath)):
                done_at = now
            if now > t_end or (done_at is not None and now - done_at > 30.0):
                if now > t_end:
                    sys.stderr.write(f"[bench supervisor] rank {rank}: attempt {k} exceeded {per_attempt_s:.0f}s, "
                                     f"killed\n")
                proc.kill()
                break
            time.sleep(0.2)
        rc = proc.wait()
        if rank == 0:
            th.join(timeout=10)
            more = k + 1 < len(attempts) and attempt_budget(time.monotonic() - t_start, deadline, cap) > 0
            verdict = "done" if printed else ("retry" if more else "giveup")
            with open(os.path.join(d, f"attempt{k}.verdict.tmp"), "w") as f:
                f.write(verdict)
            os.replace(os.path.join(d, f"attempt{k}.verdict.tmp"), os.path.join(d, f"attempt{k}.verdict"))
        else:
            verdict = _wait_file(os.path.join(d, f"attempt{k}.verdict"), 30.0)
        if verdict == "done":
            return 0
        sys.stderr.write(f"[bench supervisor] rank {rank}: attempt {k} (p2p={p2p}, graphs={graphs}) failed "
                         f"(rc={rc}); {'retrying' if verdict == 'retry' else 'giving up'} "
                         f"({time.monotonic() - t_start:.0f}s of the {deadline:.0f}s deadline used)\n")
        sys.stderr.flush()
        if verdict != "retry":
            break
    return 1


# ------------------------------------------------------------------------------ benchmark
def _plain_summary():
    """Plain forward / dX GEMM shapes per backend (ops.kernels MIPIPE_GEMM=auto timing)."""
    from mipipe.ops import kernels as K
    ch = K.plain_gemm_choices()
    if not ch:
        return None
    return {"policy": K.GEMM_BACKEND, "hipblaslt": sorted(k for k, v in ch.items() if v == "blas"),
            "mipipe": sum(1 for v in ch.values() if v == "hip")}


def run(a) -> None:
    import torch
    import torch.distributed as dist
    import mipipe  # noqa: F401
    from mipipe.engine import PipelineTrainer
    from mipipe.models.config import NativeConfig
    from mipipe.parallel.mesh import init_distributed
    from mipipe.parallel.schedules import analytic_bubble
    from mipipe.utils.fault import maybe_stall
    from mipipe.utils.metrics import Watchdog

    attempt = int(os.environ.get("MIPIPE_BENCH_ATTEMPT", "0"))
    step_to = a.step_timeout if a.step_timeout is not None else 60.0
    init_to = max(180.0, 3 * step_to)
    budget = float(os.environ.get("MIPIPE_BENCH_ATTEMPT_S", "0") or 0)
    if budget > 0:      # under the supervisor: every watchdog inside this attempt's budget
        init_to = min(init_to, max(10.0, budget - 10.0))
        step_to = min(step_to, init_to)
    describe = {"fn": lambda: "(initialising: no program yet)"}
    wd = Watchdog(init_to, describe=lambda: describe["fn"]())
    with wd.step(init_to):
        rank, world, local_rank, device = init_distributed()
        dp = a.dp
        pp = world // dp
        if pp * dp != world:
            raise SystemExit(f"--dp {dp} does not divide WORLD_SIZE={world}")
        # 128 sequences per GPU per step by default (weak scaling): one GPU runs two
        # 64-sequence microbatches (no bubble to amortise; the two microbatch lanes overlap),
        # a pipeline of P ranks 4P microbatches of 32 (1F1B bubble (P-1)/(5P-1))
        if a.mbs is None:
            a.mbs = 64 if (pp == 1 and a.microbatches is None) else 32
            m_default = 2 if pp == 1 else 4 * pp
        else:
            m_default = 4 * pp
        m = a.microbatches if a.microbatches is not None else m_default
        kw = {"vocab_size": a.vocab} if a.vocab else {}
        cfg = NativeConfig.by_name(a.model, **kw)
        gpu = device.type == "cuda"
        if a.graphs is None:
            a.graphs = 1 if gpu else 0
        dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[a.dtype or ("bf16" if gpu else "fp32")]
        trainer = PipelineTrainer(cfg, pp=pp, dp=dp, schedule=a.schedule if pp > 1 else "1F1B", n_microbatches=m,
                                  mbs=a.mbs, seq_len=a.seq, v=a.vstages, device=device,
                                  recompute=a.recompute if a.recompute == "auto" else a.recompute == "1", seed=0,
                                  split_head=False if a.no_split_head else None, graphs=bool(a.graphs) and gpu,
                                  dtype=dtype)
        describe["fn"] = trainer.runtime.describe
        gb = dp * m * a.mbs
        g = torch.Generator(device=device).manual_seed(1234 + trainer.mesh.dp_rank)
        tokens = torch.randint(0, cfg.vocab_size, (m * a.mbs, a.seq), device=device, generator=g)
        targets = torch.randint(0, cfg.vocab_size, (m * a.mbs, a.seq), device=device, generator=g)
        if a.graphs and gpu:
            trainer.capture_graphs(tokens, targets)   # setup: capture per-microbatch HIP graphs

    def sync():
        if world > 1:
            dist.barrier()
        if gpu:
            torch.cuda.synchronize()

    step_no = 0
    for _ in range(a.warmup):
        with wd.step(init_to):
            maybe_stall(rank, step_no, attempt)
            trainer.train_step(tokens, targets)
            step_no += 1
    with wd.step(init_to):
        sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        with wd.step(step_to):
            maybe_stall(rank, step_no, attempt)
            loss = trainer.train_step(tokens, targets)
            step_no += 1
    with wd.step(init_to):
        sync()
    elapsed = time.perf_counter() - t0
    with wd.step(init_to):
        if world > 1:
            t = torch.tensor([elapsed], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
    tokens_per_step = gb * a.seq
    value = tokens_per_step * a.steps / elapsed
    ms = elapsed / a.steps * 1e3

    # one extra profiled step on the same (native tape) path: measured bubble
    bubble = per_rank = None
    src = None
    if not a.no_bubble:
        with wd.step(init_to):
            sync()
            trainer.runtime.profile = True
            trainer.train_step(tokens, targets)
            trainer.runtime.profile = False
            src = trainer.runtime.last_timeline_source
            mine = torch.tensor([trainer.runtime.busy_ms(), trainer.runtime.last_step_ms], device=device,
                                dtype=torch.float64)
            if world > 1:
                allv = [torch.zeros_like(mine) for _ in range(world)]
                dist.all_gather(allv, mine)
            else:
                allv = [mine]
            busy = [float(x[0]) for x in allv]
            steps_ms = [float(x[1]) for x in allv]
            step_common = max(steps_ms)
            bubble = 1.0 - sum(busy) / (len(busy) * step_common) if step_common > 0 else None
            per_rank = [round(max(0.0, 1.0 - b / step_common), 4) for b in busy]
            if a.trace:
                from mipipe.utils.profiling import timeline_to_chrome
                timeline_to_chrome(trainer.runtime.last_timeline, f"{a.trace}.rank{rank}.json", rank)
    with wd.step(init_to):
        loss_val = None
        if trainer.is_last and loss is not None:
            loss_val = float(loss.item())
        # the loss lives on the last pipeline rank (every rank with a distributed head)
        if world > 1 and trainer.head is None:
            lv = torch.tensor([loss_val if loss_val is not None else 0.0], device=device, dtype=torch.float64)
            dist.all_reduce(lv, op=dist.ReduceOp.SUM)
            loss_val = float(lv.item()) / dp
    hbm_peak = None
    if gpu:
        with wd.step(init_to):
            hp = torch.tensor([torch.cuda.max_memory_allocated(device) / 2 ** 30], device=device, dtype=torch.float64)
            if world > 1:
                dist.all_reduce(hp, op=dist.ReduceOp.MAX)
            hbm_peak = round(float(hp.item()), 1)
    flops = cfg.flops_per_token(a.seq) * value
    rt = trainer.runtime
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "baseline_note": BASELINE_NOTE,
        "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
        "data": "synthetic uniform tokens, random-init weights",
        "bubble_fraction": None if bubble is None else round(bubble, 4),
        "bubble_per_rank": per_rank,
        "bubble_source": src,
        "analytic_bubble": round(analytic_bubble(trainer.schedule, pp, m, trainer.v), 4),
        "model_tflops_per_gpu": round(flops / world / 1e12, 1),
        "hbm_peak_gb_per_gpu": hbm_peak,   # max over ranks of the caching allocator's peak
        "attempt": attempt,
        "config": {"model": a.model, "params": cfg.n_params(), "global_batch": gb, "seq_len": a.seq,
                   "micro_batch": a.mbs, "microbatches": m, "schedule": trainer.schedule, "v": trainer.v,
                   "parallelism": f"pp{pp}" + (f"_dp{dp}" if dp > 1 else ""),
                   "layer_split": trainer.layer_ranges, "optimizer": "AdamW(fused, clip 1.0)",
                   "hip_graphs": bool(a.graphs) and gpu,
                   "microbatch_lanes": getattr(trainer, "lanes", 1),
                   "native_runner": rt.native_runner is not None,
                   "native_reason": rt.native_reason,
                   "p2p": rt.p2p.kind,
                   "p2p_channels": rt.p2p.channels if rt.p2p.kind == "native" else None,
                   "p2p_fallback": rt.p2p.fallback_reason or None,
                   "collectives": trainer.coll.kind,
                   "collective_placement": rt.coll_placement,
                   "head_zero": bool(getattr(trainer, "head_zero", False)) and trainer.head is not None,
                   "recompute": trainer.recompute,
                   "recv_arena_mb": round(rt.recv_arena_bytes / 2 ** 20, 1),
                   "plain_gemms": _plain_summary(),
                   "head": ("distributed, token chunks " + str(trainer.head_chunks)) if trainer.head is not None
                   else "last stage",
                   "head_lag": getattr(trainer, "head_lag", None),
                   "planned_efficiency": None if getattr(trainer, "planned_makespan", None) is None else
                   round(trainer.planned_ideal / trainer.planned_makespan, 3)},
    }
    if loss_val is not None:
        out["last_loss"] = round(loss_val, 4)
    if rank == 0:
        print(json.dumps(out), flush=True)
    with wd.step(init_to):
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
    wd.close()


def main():
    argv = sys.argv[1:]
    a = parse(argv)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    n = a.gpus if a.gpus is not None else world_env
    if n > 1 and world_env == 1 and "RANK" not in os.environ:
        # not launched by torch.distributed.run: launch ourselves (before touching the GPU)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", "29533"),
               os.path.abspath(__file__)] + argv
        sys.exit(subprocess.call(cmd))
    if n != world_env and world_env > 1:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE={world_env}")
    if world_env > 1 and os.environ.get("MIPIPE_BENCH_CHILD") != "1" and not a.no_supervise:
        # drop a --graphs the supervisor will set per attempt
        child_argv, skip = [], False
        for x in argv:
            if skip:
                skip = False
                continue
            if x == "--graphs":
                skip = True
                continue
            if x.startswith("--graphs="):
                continue
            child_argv.append(x)
        sys.exit(supervise(a, child_argv))
    run(a)


if __name__ == "__main__":
    main()
