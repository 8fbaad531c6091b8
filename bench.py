#!/usr/bin/env python3
"""Flagship benchmark: GPT-2 pipeline-parallel training throughput on MI355X, with the
reference's schedule comparison (GPipe vs 1F1B vs Interleaved1F1B) in the same call.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model gpt2-small]
                    [--schedule 1F1B] [--schedules all] [--ref-fp32 auto]
                    [--mbs MBS] [--seq 1024] [--microbatches M]

N GPUs = N pipeline stages (PP=N, one process per GPU); for N>1 the driver launches it
with torch.distributed.run (if launched without it, this script re-launches itself under
torch.distributed.run).  Work per GPU is fixed as N grows ("weak" scaling): every GPU
runs 128 sequences of ``seq`` tokens through all of its layers per step, so the global
batch is 128 N sequences.  A pipeline (N > 1) splits it into microbatches of 32 or 16
sequences, planned by rank 0's supervisor (engine.pick_microbatch: planned pipeline
efficiency x measured per-microbatch kernel rate; ``config.mbs_choice``); at P = 8 the
global batch is 1M tokens.
One GPU has no bubble to amortise and runs 2 microbatches of 64 (the two microbatch lanes
overlap them; profiles/r3_bench_mbs64_ab.txt).  Each timed step is a full training step:
all microbatch forwards/backwards through the lowered schedule, p2p of activations and
gradients, grad-norm clip and the fused AdamW update.

One call measures, each in a fresh child process group (so one can never cost another):
  1. the headline (``value``, ``ms_per_step``, ``config``): ``--schedule`` (auto: the best
     planned of GPipe / 1F1B / Interleaved1F1B / ZBH1, ``config.schedule_choice``);
  2. ``schedules``: GPipe, 1F1B, Interleaved1F1B (v=2) and ZBH1 on the same model, batch and
     microbatches -- tok/s, measured + analytic bubble, speedup vs GPipe, planned
     efficiency, head lag, HBM peak, p2p bytes per step (the reference's whole result,
     helper:215-220 / nb:402-433);
  3. ``reference_fp32`` (GPU default): the reference's own config -- fp32 L8 H8 d768, batch
     32 x 128, m = 4, fwd+bwd only -- through the compat API on the native fp32 kernels,
     per schedule at P = N, next to the published row of BASELINE.md (``x_vs_nb``);
  4. ``baseline_configs`` (GPU default, N = 4 / 8): BASELINE.json's named configs.
Extras only start once the headline is in and only if the time left covers them (global
deadline below); a skipped or failed extra is reported as such.

Execution path (the same at every N): per-microbatch stage compute replayed as HIP graphs,
one step recorded as a native instruction tape (csrc/runtime/stage_runner.cpp) and replayed
from C++; p2p on the native RCCL engine (one communicator + stream per direction,
csrc/comm/rccl_engine.h), pre-flight pinged at init with an in-process fallback to torch
p2p.  The JSON reports which path ran (``hip_graphs``, ``native_runner``, ``p2p``) and
what the transport carried (``p2p_bytes_per_step``, ``rccl_ranks``).

Hang safety: the pipeline program is PROVEN hang-free before it runs
(PipelineRuntime._prove), and every measurement runs in a child process under a
supervisor.  The child arms a watchdog over init, warmup, every timed step and the bubble
step (on a stall it prints the program grid + all stacks and exits non-zero); the
process-group timeout is 300 s.  If the headline fails on any rank, the supervisors retry
it in a more conservative mode (the native engine with collectives deferred to the step
end and one compute stream per rank, then torch p2p, then no HIP graphs, last every
process group on gloo) on a fresh rendezvous port; ``attempt`` / ``attempt_mode`` say which one produced the number, and
the other schedules run in that mode.  One global deadline
(MIPIPE_BENCH_DEADLINE_S, default 540 s, under the driver's 600 s) bounds everything:
each child gets at most what is left of it (and at most MIPIPE_BENCH_ATTEMPT_S, default
240 s), its watchdogs are clamped to that.  Supervisors never touch the GPU.

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

# supervisor attempts of the headline: (p2p transport, HIP graphs + native tape).  "-safe":
# the native engine with the round-4 concurrency features off -- collectives deferred to
# the step end (serial-model proof) and one compute stream per pipeline rank.  "gloo": the
# last resort when RCCL itself is unusable on the node -- every process group on gloo, p2p
# and collectives staged through host memory (slow, but a measured, labelled number:
# attempt_mode = "gloo", p2p = "gloo-staged")
ATTEMPTS = [("auto", 1), ("auto-safe", 1), ("torch", 1), ("torch", 0), ("gloo", 1)]
# the reference's three schedules (helper:215-220), measured back to back in one call
SCHEDULES = ("GPipe", "1F1B", "Interleaved1F1B")
# ... and the entries measured next to them by --schedules all: 1F1B at the
# reference's own warmup depth (P - s forwards, torch schedules.py:873-876: the distributed
# head's lag capped at 0) next to 1F1B with the planner's head lag ("1F1B+lag"), and the
# zero-bubble ZBH1.  Entry -> (schedule, extra argv).  A result is labelled by what it ran:
# "<schedule>+lag<k>" when its head lag k > 0
SCHED_VARIANTS = {"GPipe": ("GPipe", []), "1F1B": ("1F1B", ["--head-max-lag", "0"]), "1F1B+lag": ("1F1B", []),
                  "Interleaved1F1B": ("Interleaved1F1B", []), "ZBH1": ("ZBH1", [])}
ALL_SCHEDULES = ("GPipe", "1F1B", "1F1B+lag", "Interleaved1F1B", "ZBH1")
# layers of the named models (the supervisor imports nothing: model_layers); "name:L" overrides
MODEL_LAYERS = {"gpt2-tiny": 4, "gpt2": 12, "gpt2-small": 12, "gpt2-medium": 24, "gpt2-large": 36, "gpt2-xl": 48,
                "llama3": 32, "llama3-8b": 32, "llama3-1b": 16, "llama3-tiny": 4}
# the reference's 9 (L, H) configs (nb:346-349), L8 H8 first; its published rows are
# mipipe.bench.published (nb:679-732) -- imported lazily: the
# supervisor itself imports nothing that could touch HIP
REF_CONFIGS = ((8, 8), (4, 4), (4, 8), (4, 12), (8, 4), (8, 12), (12, 4), (12, 8), (12, 12))


def ref_ps(world: int) -> list:
    """Pipeline sizes of the fp32 reference phase: the P the reference published (2, 4),
    on rank subsets 0..P-1 of this launch, then P = world -- so an N = 8 record compares
    P = 2 with the P = 2 rows and P = 4 with the P = 4 rows, never P = 8 with either."""
    return [p for p in (2, 4) if p < world] + [world]


def ref_grid(a, P: int) -> list:
    """(L, H) configs the fp32 reference child at pipeline size P runs."""
    if a.ref_args != "8,8,32,128":
        L, H = (int(x) for x in a.ref_args.split(",")[:2])
        return [(L, H)]
    g = a.ref_grid or ("all" if P in (2, 4) else "l8h8")
    if g == "all":
        return list(REF_CONFIGS)
    if g == "l8h8":
        return [(8, 8)]
    return [tuple(int(x) for x in item.split(",")) for item in g.split(";") if item.strip()]


# BASELINE.json's named multi-GPU configs (configs/*.yaml), measured after everything else
# at the GPU count they name, each in its own child, only if the deadline leaves room:
# (name, extra argv, estimated child seconds beyond the headline child's wall)
BASE_CONFIGS = {
    4: [("gpt2-small 1F1B PP=4 microbatches=8 (configs/gpt2_small_1f1b_pp4.yaml)",
         ["--model", "gpt2-small", "--schedule", "1F1B", "--mbs", "16", "--microbatches", "8"], 0.0)],
    8: [("gpt2-medium Interleaved1F1B PP=8 v=2 (configs/gpt2_medium_interleaved_pp8.yaml)",
         ["--model", "gpt2-medium", "--schedule", "Interleaved1F1B", "--vstages", "2", "--mbs", "8",
          "--microbatches", "16"], 30.0),
        # selective recompute from the HBM plan: the fewest recomputed layers
        # per stage that fit (config.recompute_layers in the record), instead of every layer
        ("llama3-8b 1F1B PP=8 recompute (configs/llama3_8b_1f1b_pp8.yaml)",
         ["--model", "llama3-8b", "--schedule", "1F1B", "--mbs", "1", "--microbatches", "16", "--seq", "8192",
          "--recompute", "auto"], 120.0),
        # (BASELINE.json names recompute only for the PP = 8 config; here the HBM plan decides
        # from the schedule's real in-flight stashes -- parallel/stash.py)
        ("llama3-8b DP=2 x PP=4 recompute auto (configs/llama3_8b_dp2_pp4.yaml)",
         ["--model", "llama3-8b", "--dp", "2", "--schedule", "1F1B", "--mbs", "1", "--microbatches", "8", "--seq",
          "8192", "--recompute", "auto"], 120.0)],
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--schedule", default="auto",
                    help="the headline schedule (``value``); auto: the best planned of GPipe / 1F1B / "
                         "Interleaved1F1B (engine.pick_schedule; 1F1B at one GPU)")
    ap.add_argument("--schedules", default="all",
                    help="schedules also measured after the headline, each in a fresh child process group: "
                         "'all' (GPipe,1F1B,Interleaved1F1B,ZBH1), 'none', or a comma list")
    ap.add_argument("--ref-fp32", default="auto", choices=["auto", "0", "1"],
                    help="also time the reference's own config (fp32 L8 H8, batch 32 x 128, m=4, fwd+bwd) through "
                         "the compat API on the native fp32 path, per schedule (auto: with a GPU)")
    ap.add_argument("--base-configs", default="auto", choices=["auto", "0", "1"],
                    help="at N = 4 / 8 also measure BASELINE.json's named configs (BASE_CONFIGS) last, if time "
                         "allows (auto: on a GPU box only -- Llama-3 8B is not a CPU job)")
    ap.add_argument("--ref-args", default="8,8,32,128",
                    help="reference-config layers,heads,batch,seq (CPU tests shrink it)")
    ap.add_argument("--ref-grid", default=None,
                    help="reference (L,H) configs of the fp32 phase: 'l8h8', 'all' (the 9 of nb:346-349) or "
                         "'L,H;L,H' (default: all at P = 2 / 4, where the reference published, else L8 H8)")
    ap.add_argument("--ref-p", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--phase", default="sched", choices=["sched", "ref", "plan", "rate"], help=argparse.SUPPRESS)
    ap.add_argument("--rate-pp", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--rates", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--mbs", type=int, default=None,
                    help="sequences per microbatch (default: 64 on one GPU; with a pipeline the supervisor "
                         "plans 32 or 16 -- engine.pick_microbatch -- and 32 without it)")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--microbatches", type=int, default=None)
    ap.add_argument("--dp", type=int, default=1)
    # (not "--v": torch.distributed.run's argparse would take it for an abbreviation of
    # its --virtual-local-rank even after the script name)
    ap.add_argument("--vstages", type=int, default=None, help="virtual stages per rank (interleaved)")
    ap.add_argument("--recompute", nargs="?", const="1", default="0",
                    help="activation recompute: 1 (every layer), 0 (off), auto (selective: the fewest layers per "
                         "stage the HBM plan needs, 0 if the stash fits), or k (the first k layers of every stage)")
    ap.add_argument("--graphs", type=int, default=None,
                    help="replay per-microbatch stage compute as HIP graphs + native tape (default: on with a GPU)")
    ap.add_argument("--no-split-head", action="store_true",
                    help="keep the LM head on the last stage (default with PP>1: distributed head)")
    ap.add_argument("--no-bubble", action="store_true", help="skip the profiled bubble-measurement step")
    ap.add_argument("--trace", default=None, help="write a Chrome trace of the profiled step (per rank)")
    ap.add_argument("--step-timeout", type=float, default=None,
                    help="watchdog limit per timed step in s (default 60; 180 for init and the first steps)")
    ap.add_argument("--max-attempts", type=int, default=len(ATTEMPTS), help="supervisor attempts (headline)")
    ap.add_argument("--no-supervise", action="store_true", help="run the headline in this process (no retry, "
                                                                  "no other schedules)")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32"], help="default bf16 on GPU, fp32 on CPU")
    ap.add_argument("--vocab", type=int, default=None, help="override the vocabulary (CPU tests)")
    ap.add_argument("--head-max-lag", type=int, default=None,
                    help="cap on the distributed head's lag (extra warmup forwards; 0 = the schedule's own depth)")
    ap.add_argument("--compare-model", default="auto",
                    help="model of the schedule comparison (``schedules``): 'same', a name ('name:L' = L layers), or "
                         "auto: the headline model, unless it cannot interleave two chunks per rank at this pipeline "
                         "size (fewer than 2P layers: GPT-2 small at P = 8), then the smallest GPT-2 that can")
    return ap.parse_args(argv)


def model_layers(name: str):
    base, _, L = name.partition(":")
    return int(L) if L else MODEL_LAYERS.get(base.lower())


def model_config(name: str, vocab=None):
    """NativeConfig of ``name`` ('name:L': with L layers), vocabulary overridden by ``vocab``."""
    from mipipe.models.config import NativeConfig
    base, _, L = name.partition(":")
    kw = {"vocab_size": vocab} if vocab else {}
    if L:
        kw["n_layers"] = int(L)
    return NativeConfig.by_name(base, **kw)


def compare_model(a, pp: int) -> str:
    """The model the schedule comparison runs on (``--compare-model``): the reference's result
    is GPipe vs 1F1B vs Interleaved at the same (L, H, P) (helper:215-220), so every entry
    must be able to run the schedule it names -- interleaving needs 2P layers."""
    cm = (a.compare_model or "auto").strip()
    if cm == "same":
        return a.model
    if cm != "auto":
        return cm
    L = model_layers(a.model)
    if pp <= 1 or L is None or L >= 2 * pp:
        return a.model
    if a.model.lower().startswith("gpt2"):
        for cand in ("gpt2-medium", "gpt2-large", "gpt2-xl"):
            if MODEL_LAYERS[cand] >= 2 * pp:
                return cand
    return a.model


def _recompute_arg(v: str):
    """--recompute: "0" / "1" / "auto" / an int k (selective: the first k layers per stage)."""
    v = str(v).strip().lower()
    if v in ("auto", "selective"):
        return "auto"
    if v in ("1", "true", "on", "full"):
        return True
    if v in ("0", "false", "off", "none"):
        return False
    if v.startswith("k=") or v.isdigit():
        return int(v[2:] if v.startswith("k=") else v)
    raise SystemExit(f"--recompute: 0, 1, auto or an integer, not {v!r}")


def extra_schedules(a) -> list:
    s = (a.schedules or "none").strip()
    if s.lower() in ("none", "0", ""):
        names = []
    elif s.lower() == "all":
        names = list(ALL_SCHEDULES)
    else:
        names = [x.strip() if x.strip() in SCHED_VARIANTS else _canon(x) for x in s.split(",") if x.strip()]
    return names


def _canon(name: str) -> str:
    """Schedule name -> canonical (the supervisor imports nothing that could touch HIP)."""
    key = name.replace("_", "").replace("-", "").lower()
    table = {"gpipe": "GPipe", "1f1b": "1F1B", "interleaved": "Interleaved1F1B", "interleaved1f1b": "Interleaved1F1B",
             "zbh1": "ZBH1", "zbv": "ZBV", "loopedbfs": "LoopedBFS", "auto": "auto"}
    if key not in table:
        raise SystemExit(f"unknown schedule {name!r}")
    return table[key]


def ref_fp32_on(a) -> bool:
    if a.ref_fp32 != "auto":
        return a.ref_fp32 == "1"
    import shutil
    # a GPU box (the supervisor never initialises HIP: device nodes / rocminfo only)
    return os.path.exists("/dev/kfd") and shutil.which("rocminfo") is not None


# ------------------------------------------------------------------------------ supervisor
def _attempt_dir() -> str:
    # one node (--nnodes=1): every rank's supervisor is a child of the same launcher agent
    # (one process without a launcher: this process's own id)
    owner = os.getppid() if int(os.environ.get("WORLD_SIZE", "1")) > 1 else os.getpid()
    d = os.path.join(os.environ.get("TMPDIR", "/tmp"),
                     f"mipipe_bench_{owner}_{os.environ.get('MASTER_PORT', '0')}")
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


def _publish(path: str, text: str) -> None:
    with open(path + ".tmp", "w") as f:
        f.write(text)
    os.replace(path + ".tmp", path)


DEADLINE_S = 540.0       # all attempts together (the driver kills the bench at 600 s)
ATTEMPT_CAP_S = 240.0    # one attempt at most
MIN_ATTEMPT_S = 30.0     # no attempt starts with less than this left


def attempt_budget(elapsed: float, deadline: float = DEADLINE_S, cap: float = ATTEMPT_CAP_S) -> float:
    """Seconds the next attempt may run (0: none may start) -- what is left of the global
    deadline, less a 5 s margin for killing a child, capped per attempt."""
    left = deadline - elapsed - 5.0
    return 0.0 if left < MIN_ATTEMPT_S else min(cap, left)


def extra_budget(kind: str, left: float, cap: float, head_wall: float, ref_wall=None) -> tuple:
    """(seconds the next non-headline child may run, 0 = skip it; its estimated need).
    The need is the headline child's wall time + 25 % + 10 s (same model, one attempt) or
    the last reference child's; the child is killed at twice that (>= 90 s), and never
    later than 10 s before the global deadline -- so however the extras end, the whole
    run stays inside it."""
    est = head_wall * 1.25 + 10.0
    if kind.startswith("ref"):      # "ref:<runs>": one child runs <runs> (L, H, schedule) configs
        runs = int(kind.split(":", 1)[1]) if ":" in kind else 3
        # ~3 s per config on a GPU once a child has measured it (20 s for its start-up;
        # MIPIPE_BENCH_REF_RUN_S: the per-config guess before any child measured one)
        est = 20.0 + runs * (ref_wall if ref_wall else float(os.environ.get("MIPIPE_BENCH_REF_RUN_S", "3")))
    if kind.startswith("base"):     # "base:<extra seconds>"
        est = head_wall * 1.25 + 10.0 + float(kind.split(":", 1)[1] if ":" in kind else 0.0)
    b = min(cap, left - 10.0)
    if kind.startswith("ref"):
        # a reference child truncates its grid to its budget (run_ref): it only needs room
        # for the first config's three schedules
        if b < max(MIN_ATTEMPT_S, 20.0 + 3 * (ref_wall if ref_wall else 3.0)):
            return 0.0, est
        return min(b, max(2.0 * est, 90.0)), est
    if b < max(MIN_ATTEMPT_S, est):
        return 0.0, est
    return min(b, max(2.0 * est, 90.0)), est


def child_env(base: dict, p2p: str, attempt: int, port: int, budget: float, res_path: str) -> dict:
    """Environment of one supervised child: its attempt mode (ATTEMPTS), a fresh rendezvous
    port, its time budget and where rank 0 writes the result."""
    env = dict(base, MIPIPE_BENCH_CHILD="1", MIPIPE_P2P=p2p.split("-")[0], MIPIPE_BENCH_ATTEMPT=str(attempt),
               MASTER_PORT=str(port), MIPIPE_BENCH_ATTEMPT_S=f"{budget:.0f}", MIPIPE_BENCH_RESULT=res_path,
               MIPIPE_BENCH_MODE=p2p)
    if p2p == "gloo":
        env.update(MIPIPE_DIST_BACKEND="gloo", MIPIPE_P2P="auto")
    if p2p.endswith("-safe"):
        # the second attempt drops what a first multi-GPU run has never exercised: collective
        # overlap, lanes at PP > 1 and receive-only posts ahead of the compute (recv-early)
        env.update(MIPIPE_COLL_OVERLAP="0", MIPIPE_PP_LANES="0", MIPIPE_RECV_EARLY="0")
    env.pop("TORCHELASTIC_USE_AGENT_STORE", None)   # fresh rendezvous store per child
    return env


def plan_phases(a, argv) -> list:
    """The fixed, rank-independent list of child runs: (tag, kind, argv, schedule).  The
    headline's attempts first, then every other schedule of ``--schedules`` on the same
    model/config, then the reference's fp32 config per schedule."""
    tags = [(f"h{k}", "headline", list(argv), a.schedule) for k in range(max(1, a.max_attempts))]
    # every comparison entry gets a slot (on the comparison model: compare_model); the one the
    # headline ran (known once it is in: same model, planned lag) is skipped.  One GPU has no
    # pipeline and no head lag: "1F1B+lag" would repeat "1F1B"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    pp = max(1, world // max(1, a.dp))
    cmodel = compare_model(a, pp)
    for s in extra_schedules(a):
        sched, extra = SCHED_VARIANTS.get(s, (s, []))
        if s == "1F1B+lag" and pp == 1:
            continue
        margv = [] if cmodel == a.model else ["--model", cmodel]
        tags.append((f"x_{s}", "sched", list(argv) + ["--schedule", sched] + extra + margv, s))
    if ref_fp32_on(a):
        world = int(os.environ.get("WORLD_SIZE", "1"))
        for P in ref_ps(world):
            # one child per pipeline size runs every (L, H) config x schedule of its grid
            # (one process group, one set of RCCL communicators), ranks >= P sit it out
            tags.append((f"r{P}", "ref", list(argv) + ["--phase", "ref", "--ref-p", str(P)], f"P{P}"))
    if (a.base_configs == "1") or (a.base_configs == "auto" and ref_fp32_on(argparse.Namespace(ref_fp32="auto"))):
        world = int(os.environ.get("WORLD_SIZE", "1"))
        for k, (name, extra, _) in enumerate(BASE_CONFIGS.get(world, [])):
            tags.append((f"b{k}", "base", list(argv) + ["--dp", "1"] + extra, name))
    return tags


def supervise(a, argv) -> int:
    """Run every measurement in a child process (module docstring): the headline with up to
    ``--max-attempts`` increasingly conservative attempts, then -- only once the headline
    is in -- the other schedules and the reference's fp32 config, one fresh child process
    group each, each only if the time left in the global deadline covers it (estimated from
    the headline child's wall time).  A failing or hung extra is recorded as such and never
    costs the headline.  Rank 0 decides every step and publishes it in a per-launch
    directory (``<tag>.go``: "go <budget_s> <p2p> <graphs> <attempt>" | "skip"); the other
    ranks follow.  Rank 0 prints ONE JSON line at the end.  Never initialises the GPU."""
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

    def left() -> float:
        return deadline - (time.monotonic() - t_start)

    def run_child(j, tag, child_argv, p2p, graphs, attempt, budget, sub_world=None):
        res_path = os.path.join(d, f"{tag}.json")
        env = child_env(os.environ, p2p, attempt, base_port + 1 + j, budget, res_path)
        if sub_world is not None:
            # a pipeline on ranks 0..sub_world-1 of this launch (one GPU each, LOCAL_RANK kept)
            env.update(WORLD_SIZE=str(sub_world), LOCAL_WORLD_SIZE=str(sub_world))
        cmd = [sys.executable, os.path.abspath(__file__)] + child_argv + ["--graphs", str(graphs)]
        t0 = time.monotonic()
        proc = subprocess.Popen(cmd, env=env)
        current["proc"] = proc
        t_end = t0 + budget
        done_path = os.path.join(d, f"{tag}.done")
        done_at = None
        # wait for the child; once the result is in (rank 0's child wrote it), a child still
        # tearing down gets a grace period, then is killed
        while proc.poll() is None:
            now = time.monotonic()
            if done_at is None and os.path.exists(res_path if rank == 0 else done_path):
                done_at = now
            if now > t_end or (done_at is not None and now - done_at > 30.0):
                if now > t_end:
                    sys.stderr.write(f"[bench supervisor] rank {rank}: {tag} exceeded {budget:.0f}s, killed\n")
                proc.kill()
                break
            time.sleep(0.2)
        rc = proc.wait()
        current["proc"] = None
        res = None
        if rank == 0 and os.path.exists(res_path):
            with open(res_path) as f:
                res = json.loads(f.read())
            _publish(done_path, "1")
        elif rank == 0 and os.path.exists(res_path + ".partial"):
            with open(res_path + ".partial") as f:
                res = json.loads(f.read())    # killed at its budget: what it finished
            res["killed_at_budget_s"] = round(budget)
        return rc, res, time.monotonic() - t0

    # --mbs auto (no --mbs / --microbatches given, PP > 1): rank 0 plans the microbatch size
    # in a CPU-only child (engine.pick_microbatch) and every rank's children get it
    mbs_plan = None
    pp = max(1, int(os.environ.get("WORLD_SIZE", "1")) // max(1, a.dp))
    if a.mbs is None and a.microbatches is None and pp > 1 and os.environ.get("MIPIPE_BENCH_MBS", "auto") == "auto":
        plan_path = os.path.join(d, "mbs.plan")
        if rank == 0:
            # the per-GPU kernel rate at each candidate microbatch size, measured for THIS
            # model's per-rank shapes on GPU 0 (engine.rate_probe_config; a GPU box only)
            rates = None
            if ref_fp32_on(argparse.Namespace(ref_fp32="auto")) and os.environ.get("MIPIPE_BENCH_RATES", "1") != "0":
                rates = rate_probe_child(argv, pp, min(120.0, max(10.0, left() - 360.0)))
            # (the first `import torch` on a fresh box can take 1-2 minutes)
            plan_argv = list(argv) + (["--rates", json.dumps(rates["rates"])] if rates and "rates" in rates else [])
            mbs_plan = plan_microbatch_child(plan_argv, min(150.0, max(10.0, left() - 300.0)))
            if rates is not None:
                mbs_plan["rate_probe"] = rates
            _publish(plan_path, json.dumps(mbs_plan))
        else:
            txt = _wait_file(plan_path, 210.0)
            mbs_plan = json.loads(txt) if txt else None
        if mbs_plan and mbs_plan.get("mbs"):
            argv = list(argv) + ["--mbs", str(mbs_plan["mbs"]), "--microbatches", str(mbs_plan["microbatches"])]
    phases = plan_phases(a, argv)
    walls = {"plan": round(time.monotonic() - t_start, 1)}
    results = {}
    headline = None
    head_wall = None
    head_mode = attempts[0] + (0,)
    ref_wall = None
    n_head = len([p for p in phases if p[1] == "headline"])
    for j, (tag, kind, child_argv, sched) in enumerate(phases):
        go_path = os.path.join(d, f"{tag}.go")
        if rank == 0:
            decision = "skip"
            if kind == "headline":
                k = int(tag[1:])
                b = attempt_budget(deadline - left(), deadline, cap)
                if headline is None and k < len(attempts) and b > 0:
                    decision = f"go {b:.0f} {attempts[k][0]} {attempts[k][1]} {k}"
            elif (headline is not None and kind == "sched" and SCHED_VARIANTS.get(sched, (sched, []))[1] == []
                  and SCHED_VARIANTS.get(sched, (sched, []))[0] == headline["config"]["schedule"]
                  and compare_model(a, pp) == a.model and a.head_max_lag is None):
                pass        # the headline's own schedule (same model, planned lag): already measured
            elif headline is not None:
                kb = kind
                if kind == "base":
                    world = int(os.environ.get("WORLD_SIZE", "1"))
                    kb = f"base:{BASE_CONFIGS[world][int(tag[1:])][2]}"
                elif kind == "ref":
                    kb = f"ref:{len(ref_grid(a, int(tag[1:]))) * len(SCHEDULES)}"
                b, est = extra_budget(kb, left(), cap, head_wall, ref_wall)
                if b > 0:
                    decision = f"go {b:.0f} {head_mode[0]} {head_mode[1]} {head_mode[2]}"
                else:
                    results[tag] = {"skipped": f"time: {left():.0f}s left of the {deadline:.0f}s deadline, "
                                               f"~{est:.0f}s needed"}
            _publish(go_path, decision)
        else:
            decision = _wait_file(go_path, max(60.0, left() + 60.0)) or "skip"
        if not decision.startswith("go"):
            continue
        _, b, p2p, graphs, att = decision.split()
        if kind == "headline" and int(att) >= 1 and _canon(a.schedule) == "auto":
            # a planned schedule that failed once is not retried: the later attempts run 1F1B,
            # the schedule every multi-rank test runs
            child_argv = list(child_argv) + ["--schedule", "1F1B"]
        sub = None
        if kind == "ref":
            sub = int(tag[1:])
            if rank >= sub:
                continue        # a pipeline on ranks 0..P-1: this rank sits it out
            sub = sub if sub < int(os.environ.get("WORLD_SIZE", "1")) else None
        rc, res, wall = run_child(j, tag, child_argv, p2p, int(graphs), int(att), float(b), sub)
        walls[tag] = round(wall, 1)
        if rank != 0:
            continue
        if kind == "headline":
            if res is not None:
                headline, head_wall, head_mode = res, wall, (p2p, int(graphs), int(att))
            else:
                more = (int(tag[1:]) + 1 < min(n_head, len(attempts))
                        and attempt_budget(deadline - left(), deadline, cap) > 0)
                sys.stderr.write(f"[bench supervisor] headline attempt {tag[1:]} (p2p={p2p}, graphs={graphs}) "
                                 f"failed (rc={rc}); {'retrying' if more else 'giving up'} "
                                 f"({deadline - left():.0f}s of the {deadline:.0f}s deadline used)\n")
        else:
            if kind == "ref":
                # per (L, H, schedule) run of the last reference child, for the next one's estimate
                n_runs = len(ref_grid(a, int(tag[1:]))) * len(SCHEDULES)
                ref_wall = (wall * 1.25 + 5) / max(1, n_runs)
            results[tag] = res if res is not None else {"error": f"child exited rc={rc} without a result "
                                                                 f"after {wall:.0f}s"}
    final_path = os.path.join(d, "final")
    if rank != 0:
        return 0 if _wait_file(final_path, max(60.0, left() + 60.0)) == "ok" else 1
    _publish(final_path, "ok" if headline is not None else "fail")
    if headline is None:
        return 1
    out = merge_results(headline, results, a)
    if mbs_plan is not None:
        out.setdefault("config", {})["mbs_choice"] = mbs_plan
    out["supervisor_walls_s"] = dict(walls, total=round(time.monotonic() - t_start, 1))
    print(json.dumps(out), flush=True)
    return 0


def plan_microbatch_child(argv, timeout_s: float) -> dict:
    """Run ``bench.py --phase plan`` (pure planning, no GPU) and return its JSON, or
    {"error": ...} -- the children then keep the fixed default (32 sequences)."""
    cmd = [sys.executable, os.path.abspath(__file__)] + list(argv) + ["--phase", "plan"]
    env = dict(os.environ, MIPIPE_BENCH_CHILD="1")
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout_s)
        lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode == 0 and lines:
            return json.loads(lines[-1])
        return {"error": f"plan child rc={r.returncode}: {r.stderr[-300:]}"}
    except subprocess.TimeoutExpired:
        return {"error": f"plan child exceeded {timeout_s:.0f}s"}


def rate_probe_child(argv, pp: int, timeout_s: float) -> dict:
    """Run ``bench.py --phase rate`` (one process, GPU 0) and return its JSON, or
    {"error": ...} -- the planner then uses its GPT-2-small table."""
    cmd = [sys.executable, os.path.abspath(__file__)] + list(argv) + ["--phase", "rate", "--rate-pp", str(pp)]
    env = dict(os.environ, MIPIPE_BENCH_CHILD="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1")
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout_s)
        lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode == 0 and lines:
            return json.loads(lines[-1])
        return {"error": f"rate child rc={r.returncode}: {r.stderr[-300:]}"}
    except subprocess.TimeoutExpired:
        return {"error": f"rate child exceeded {timeout_s:.0f}s"}


def run_rate(a) -> None:
    """--phase rate: tokens/s of one GPU running the per-rank work of a ``--rate-pp``-stage
    pipeline of the model (engine.rate_probe_config: L / P layers, V / P vocabulary) at each
    candidate microbatch size -- 1F1B, 4 microbatches on the default lanes, HIP graphs, 2
    warmup + 5 timed steps each."""
    import torch
    import mipipe  # noqa: F401
    from mipipe.engine import PipelineTrainer, rate_probe_config
    from mipipe.models.config import NativeConfig
    pp = max(1, a.rate_pp or 1)
    cfg = rate_probe_config(model_config(a.model, a.vocab), pp)
    gpu = torch.cuda.is_available()
    dev = torch.device("cuda", 0) if gpu else torch.device("cpu")
    t0 = time.monotonic()
    rates = {}
    for mbs in (32, 16):
        m = 4
        tr = PipelineTrainer(cfg, pp=1, schedule="1F1B", n_microbatches=m, mbs=mbs, seq_len=a.seq, device=dev,
                             seed=0, graphs=gpu)
        g = torch.Generator(device=dev).manual_seed(5)
        x = torch.randint(0, cfg.vocab_size, (m * mbs, a.seq), device=dev, generator=g)
        y = torch.randint(0, cfg.vocab_size, (m * mbs, a.seq), device=dev, generator=g)
        if gpu:
            tr.capture_graphs(x, y)
        for _ in range(2):
            tr.train_step(x, y)
        if gpu:
            torch.cuda.synchronize()
        t = time.perf_counter()
        n = 5
        for _ in range(n):
            tr.train_step(x, y)
        if gpu:
            torch.cuda.synchronize()
        rates[mbs] = round(m * mbs * a.seq * n / (time.perf_counter() - t), 1)
        del tr
        if gpu:
            torch.cuda.empty_cache()
    print(json.dumps({"rates": rates, "probe_model": {"n_layers": cfg.n_layers, "vocab": cfg.vocab_size, "pp": pp},
                      "probe_s": round(time.monotonic() - t0, 1)}), flush=True)


def run_plan(a) -> None:
    """--phase plan: the microbatch size for the supervisor (never touches the GPU)."""
    import mipipe  # noqa: F401
    from mipipe.engine import pick_microbatch
    from mipipe.models.config import NativeConfig
    world = int(os.environ.get("WORLD_SIZE", "1"))
    pp = max(1, world // max(1, a.dp))
    cfg = model_config(a.model, a.vocab)
    t0 = time.monotonic()
    rates = json.loads(a.rates) if a.rates else None
    mbs, m, scores = pick_microbatch(cfg, pp, a.seq, 128 * pp, rates=rates)
    print(json.dumps({"mbs": mbs, "microbatches": m, "scores": {str(k): v for k, v in scores.items()},
                      "plan_s": round(time.monotonic() - t0, 1)}), flush=True)


def _sched_entry(r: dict) -> dict:
    if "error" in r or "skipped" in r:
        return r
    keys = ("value", "ms_per_step", "bubble_fraction", "bubble_per_rank", "analytic_bubble", "hbm_peak_gb_per_gpu",
            "hbm_reserved_peak_gb_per_gpu", "hbm_device_used_gb_per_gpu", "model_tflops_per_gpu", "p2p_bytes_per_step",
            "rccl_ranks", "attempt", "stash_slots_per_rank")
    out = {"tok_s": r.get("value")}
    out.update({k: r.get(k) for k in keys if k != "value" and k in r})
    c = r.get("config", {})
    for k in ("model", "schedule", "v", "microbatches", "micro_batch", "head_lag", "head_max_lag", "planned_efficiency",
              "native_runner", "p2p", "layer_split", "microbatch_lanes"):
        if k in c:
            out[k] = c[k]
    return out


def merge_reference(refs: dict, world: int, a) -> dict:
    """``reference_fp32``: every measured (L, H, P, schedule) row with its speedup vs GPipe at
    the same (L, H, P), the published row of the SAME (L, H, P, schedule) where the
    reference has one (P = 2 / 4: ``nb_row``, ``x_vs_nb``), the per-P summary, and --
    for compatibility -- ``per_schedule``: L8 H8 at P = N."""
    rows, status = [], {}
    for tag, r in sorted(refs.items(), key=lambda kv: int(kv[0][1:])):
        P = int(tag[1:])
        if "rows" not in r:
            status[f"P{P}"] = r           # error / skipped
            continue
        status[f"P{P}"] = {"complete": r.get("complete"), "configs": len(r["rows"]) // len(SCHEDULES),
                           "wall_s": r.get("wall_s")}
        rows.extend(r["rows"])
    gp = {(x["L"], x["H"], x["P"]): x["tok_s"] for x in rows if x["schedule"] == "GPipe" and x.get("tok_s")}
    for x in rows:
        g = gp.get((x["L"], x["H"], x["P"]))
        if g:
            x["speedup_vs_gpipe"] = round(x["tok_s"] / g, 4)
    summary = {}
    for P in sorted({x["P"] for x in rows}):
        xs = [x["x_vs_nb"] for x in rows if x["P"] == P and "x_vs_nb" in x]
        e = {"rows": sum(1 for x in rows if x["P"] == P)}
        if xs:
            xs = sorted(xs)
            e.update(x_vs_nb_min=xs[0], x_vs_nb_median=xs[len(xs) // 2], x_vs_nb_max=xs[-1], published_rows=len(xs))
        else:
            e["published_rows"] = 0
            e["note"] = "the reference published P = 2 and 4 only (nb:679-732)"
        summary[f"P{P}"] = e
    per_schedule = {x["schedule"]: x for x in rows if (x["L"], x["H"], x["P"]) == (8, 8, world)}
    okr = [x["tok_s"] for x in per_schedule.values() if x.get("tok_s")]
    return {"config": "reference ModelArgs L x H d768 vocab 10000, batch {2} x seq {3}, m=4 (m=P for one stage "
                      "per rank at P > 4), fp32, fwd+bwd only, dropout 0.1 (helper:23-55, :98-143, :214); "
                      "P < N on ranks 0..P-1".format(*a.ref_args.split(",")),
            "status": status, "summary": summary, "rows": rows, "per_schedule": per_schedule,
            "tok_s": max(okr, default=None)}


def merge_results(headline: dict, results: dict, a) -> dict:
    """The headline's JSON line + ``schedules`` (every measured schedule of the comparison
    model at the same microbatches, the headline's own included when it ran that model, each
    labelled by what it ran: ``<schedule>+lag<k>`` with a head lag) + ``reference_fp32`` +
    ``baseline_configs``."""
    out = dict(headline)
    world = headline.get("n_gpus", 1)
    pp = max(1, world // max(1, getattr(a, "dp", 1) or 1))
    cmodel = compare_model(a, pp) if hasattr(a, "compare_model") else headline["config"].get("model")
    sched = {}

    def label(e, fallback):
        # what the entry ran: "<schedule>+lag<k>" when its distributed head ran k extra
        # warmup forwards (VERDICT r5 #1c), else the schedule's name
        if "tok_s" not in e or not e.get("schedule"):
            return fallback
        lag = e.get("head_lag") or 0
        return e["schedule"] + (f"+lag{lag}" if lag else "")

    def put(key, e):
        while key in sched:          # e.g. the planner chose lag 0 for "1F1B+lag"
            key += " (planned)"
        sched[key] = e
    if cmodel == headline["config"].get("model"):
        e = _sched_entry(headline)
        put(label(e, headline["config"]["schedule"]), e)
    for tag, r in results.items():
        if tag.startswith("x_"):
            e = _sched_entry(r)
            put(label(e, tag[2:]), e)
    out["schedules"] = sched
    out["schedules_model"] = cmodel
    if cmodel != headline["config"].get("model"):
        out["schedules_note"] = (f"{headline['config'].get('model')} cannot interleave two chunks per rank at P = {pp} "
                                 f"(fewer than 2P layers): the comparison runs on {cmodel}, same microbatches for "
                                 "every schedule")
    ok = {k: v for k, v in sched.items() if "tok_s" in v and v["tok_s"]}
    gp = next((v for k, v in ok.items() if k.startswith("GPipe")), None)
    if gp is not None:
        for k, v in ok.items():
            v["speedup_vs_gpipe"] = round(v["tok_s"] / gp["tok_s"], 4)
    refs = {tag: r for tag, r in results.items() if tag.startswith("r") and tag[1:].isdigit()}
    if refs:
        out["reference_fp32"] = merge_reference(refs, headline["n_gpus"], a)
    base = {}
    for tag, r in results.items():
        if tag.startswith("b") and tag[1:].isdigit() and world in BASE_CONFIGS:
            name = BASE_CONFIGS[world][int(tag[1:])][0]
            e = _sched_entry(r)
            if "tok_s" in e:
                c = r.get("config", {})
                e.update({k: c.get(k) for k in ("model", "schedule", "v", "parallelism", "micro_batch", "microbatches",
                                                 "seq_len", "recompute", "recompute_layers", "global_batch")})
            base[name] = e
    if base:
        out["baseline_configs"] = base
    return out


# ------------------------------------------------------------------------------ benchmark
def emit(out: dict, partial: bool = False) -> None:
    """Rank 0's result: into the supervisor's result file (MIPIPE_BENCH_RESULT), else stdout.
    ``partial``: progress of a child that may still be killed at its budget (the supervisor
    reads it only if the final result never came; it does not mark the child done)."""
    path = os.environ.get("MIPIPE_BENCH_RESULT")
    if partial and not path:
        return
    if path:
        _publish(path + (".partial" if partial else ""), json.dumps(out))
    else:
        print(json.dumps(out), flush=True)


def _concurrency_record(trainer) -> dict:
    """One rank's live concurrency features: the queue probe's verdict (comm streams on
    hardware queues of their own -> collectives overlap the flush; the shared pairs if not),
    the RCCL communicators this rank opened (pipeline channels, DP, tied embedding), its
    microbatch lanes and p2p channels."""
    rt = trainer.runtime
    rep = getattr(rt, "queue_report", None)
    probe = None
    if rep is not None:
        probe = rep.get("forced") or rep.get("gloo") or ("independent" if rep.get("independent") else
                                                         "shared: " + ",".join(rep.get("shared", [])[:4]))
    eng = getattr(rt.p2p, "engine", None)
    comms = (int(eng.channels) if eng is not None else 0)
    for name in ("dp_engine", "embed_engine"):
        e = getattr(trainer.coll, name, None)
        comms += int(e.channels) if e is not None else 0
    au = getattr(trainer, "comm_audit", None)
    mp = getattr(trainer, "memory_plan", None) or {}
    return {"queue_probe": probe, "rccl_communicators": comms, "lanes": int(getattr(trainer, "lanes", 1)),
            "stash_slots": {str(k): v for k, v in mp.get("stash_slots", {}).items()},
            "p2p_channels": int(getattr(rt.p2p, "channels", 1)), "collective_placement": rt.coll_placement,
            # first-step cross-rank check of the issued p2p order and collective sequences
            "comm_audit": None if au is None else ((f"ok ({au['entries']} groups, p2p {au.get('p2p', 'audited')})")
                                                  if au["ok"] else au["problems"])}


def _memory_plan_summary(trainer):
    """This rank's HBM plan (engine.plan_recompute): the stash slots per local stage that the
    schedule keeps alive (parallel/stash.py) and the planned bytes with / without recompute."""
    p = getattr(trainer, "memory_plan", None)
    if not p:
        return None
    return {"stash_slots": {str(k): v for k, v in p.get("stash_slots", {}).items()},
            "planned_gb_no_recompute": round(p["bytes_no_recompute"] / 1e9, 1),
            "planned_gb_recompute": round(p["bytes_recompute"] / 1e9, 1),
            "recompute_needed": bool(p["recompute"])}


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
        cfg = model_config(a.model, a.vocab)
        planned = {}
        plan_details = {}
        was_auto = _canon(a.schedule) == "auto"
        if was_auto:
            from mipipe.engine import pick_schedule
            a.schedule, planned = pick_schedule(cfg, pp, m, a.mbs, a.seq, details=plan_details)
        gpu = device.type == "cuda"
        if a.graphs is None:
            a.graphs = 1 if gpu else 0
        dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[a.dtype or ("bf16" if gpu else "fp32")]
        trainer = PipelineTrainer(cfg, pp=pp, dp=dp, schedule=a.schedule, n_microbatches=m,
                                  mbs=a.mbs, seq_len=a.seq, v=a.vstages, device=device,
                                  recompute=_recompute_arg(a.recompute), seed=0,
                                  split_head=False if a.no_split_head else None, graphs=bool(a.graphs) and gpu,
                                  dtype=dtype, head_max_lag=a.head_max_lag)
        describe["fn"] = trainer.describe
        gb = dp * m * a.mbs
        g = torch.Generator(device=device).manual_seed(1234 + trainer.mesh.dp_rank)
        tokens = torch.randint(0, cfg.vocab_size, (m * a.mbs, a.seq), device=device, generator=g)
        targets = torch.randint(0, cfg.vocab_size, (m * a.mbs, a.seq), device=device, generator=g)
        if a.graphs and gpu:
            trainer.capture_graphs(tokens, targets)   # setup: capture per-microbatch HIP graphs
        if gpu:
            # HBM peaks from here on: the training steps, not the setup's eager step
            torch.cuda.reset_peak_memory_stats(device)

    def sync():
        if world > 1:
            dist.barrier()
        if gpu:
            torch.cuda.synchronize()

    step_no = 0
    for w in range(a.warmup):
        # the first step records the native tape; later warmups replay it (a hang there is
        # caught in 90 s, not the init limit)
        with wd.step(init_to if w == 0 else min(init_to, max(step_to, 90.0))):
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
    hbm_peak = hbm_reserved = hbm_used = None
    if gpu:
        with wd.step(init_to):
            # allocated peak (what live tensors held), reserved peak (what the caching allocator
            # and the HIP-graph pools held: a graph pool keeps its freed blocks reserved), and the
            # device's used bytes (mem_get_info: also RCCL buffers, code objects, workspaces)
            free, total = torch.cuda.mem_get_info(device)
            hp = torch.tensor([torch.cuda.max_memory_allocated(device) / 2 ** 30,
                               torch.cuda.max_memory_reserved(device) / 2 ** 30, (total - free) / 2 ** 30],
                              device=device, dtype=torch.float64)
            if world > 1:
                dist.all_reduce(hp, op=dist.ReduceOp.MAX)
            hbm_peak, hbm_reserved, hbm_used = (round(float(x), 1) for x in hp.tolist())
    flops = cfg.flops_per_token(a.seq) * value
    rt = trainer.runtime
    with wd.step(init_to):
        # the record proves what the transport carried: pipeline bytes sent per step (all
        # ranks) and the ranks of the native RCCL communicators (pipeline, DP)
        pb = torch.tensor([float(rt.p2p_send_bytes())], device=device, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(pb, op=dist.ReduceOp.SUM)
        p2p_bytes = int(pb.item())
        eng = getattr(rt.p2p, "engine", None)
        rccl_ranks = {"pp": int(eng.nranks) if eng is not None else None,
                      "dp": int(trainer.coll.dp_engine.nranks) if getattr(trainer.coll, "dp_engine", None)
                      is not None else None}
        # which concurrency features were live on EVERY rank (VERDICT r4 #6c): this rank's
        # hardware-queue probe verdict, the RCCL communicators it opened, its lanes
        conc = _concurrency_record(trainer)
        if world > 1:
            allc = [None] * world
            # over the gloo control group (host objects; no device tensors on the RCCL group)
            dist.all_gather_object(allc, conc, group=trainer.mesh.world_ctrl)
        else:
            allc = [conc]
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
        # max over ranks, GiB, over the training steps after setup: the caching allocator's
        # RESERVED peak (what the device holds: HIP-graph pools keep freed blocks reserved --
        # the allocated counter drops when a capture frees them), its allocated peak, and the
        # device's used bytes at the end (mem_get_info)
        "hbm_peak_gb_per_gpu": hbm_reserved,
        "hbm_reserved_peak_gb_per_gpu": hbm_reserved,
        "hbm_allocated_peak_gb_per_gpu": hbm_peak,
        "hbm_device_used_gb_per_gpu": hbm_used,
        "attempt": attempt,
        "attempt_mode": os.environ.get("MIPIPE_BENCH_MODE", "in-process"),
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
                   "dp_reduce_dtype": ("bf16" if getattr(trainer.coll, "dp_reduce_dtype", None) == torch.bfloat16
                                       else "f32") if dp > 1 else None,
                   "head_zero": bool(getattr(trainer, "head_zero", False)) and trainer.head is not None,
                   "recompute": trainer.recompute,
                   "recompute_layers": getattr(trainer, "recompute_layers", None),
                   "memory_plan": _memory_plan_summary(trainer),
                   "recv_arena_mb": round(rt.recv_arena_bytes / 2 ** 20, 1),
                   "plain_gemms": _plain_summary(),
                   "head": ("distributed, token chunks " + str(trainer.head_chunks)) if trainer.head is not None
                   else "last stage",
                   "head_lag": getattr(trainer, "head_lag", None),
                   "head_max_lag": a.head_max_lag,
                   "planned_efficiency": None if getattr(trainer, "planned_makespan", None) is None else
                   round(trainer.planned_ideal / trainer.planned_makespan, 3),
                   "schedule_choice": ({"auto": {k: round(v_, 3) for k, v_ in planned.items()}, "plans": plan_details}
                                       if planned else ("auto (one GPU: 1F1B)" if was_auto else "given"))},
    }
    if loss_val is not None:
        out["last_loss"] = round(loss_val, 4)
    out["p2p_bytes_per_step"] = p2p_bytes
    out["rccl_ranks"] = rccl_ranks
    out["per_rank_concurrency"] = allc
    # every rank's stash slots per local stage (parallel/stash.py plan of its compute order)
    out["stash_slots_per_rank"] = [c.get("stash_slots") for c in allc]
    if rank == 0:
        emit(out)
    with wd.step(init_to):
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
    wd.close()


def run_ref(a) -> None:
    """The reference's own workload (helper:150-235 with nb:306's batch 32 x seq 128, m = 4,
    fwd+bwd only, no optimizer step) through the compat API on the native path at the
    reference's precision (fp32 kernels), on a pipeline of P = ``--ref-p`` ranks (0..P-1 of
    the launch), every schedule x every (L, H) config of ``ref_grid`` in ONE process group
    (one set of RCCL communicators, reused by every schedule).  Timing as the reference
    (wall clock over ``--steps`` steps after ``--warmup``; L8 H8 with the bench's step
    counts, the other configs with the reference's own 2 warmup + 5 timed steps, nb:372)
    and also max over ranks; plus the measured and analytic bubble.  Rank 0 re-publishes
    the rows after every config, and stops starting new configs when 80 % of the child's
    time budget is used (``complete`` says whether the whole grid ran)."""
    import gc
    import torch
    import torch.distributed as dist
    import mipipe  # noqa: F401
    from mipipe.bench.compat import native_reference_schedule, run_train_iterations, stages_per_worker
    from mipipe.bench.published import published, SOURCE_LINE
    from mipipe.models.ref_transformer import ModelArgs, Transformer, manual_model_split, tokenwise_loss_fn
    from mipipe.parallel.api import get_schedule_class
    from mipipe.parallel.comm import P2P
    from mipipe.parallel.mesh import init_distributed
    from mipipe.utils.metrics import Watchdog

    t_start = time.monotonic()
    budget = float(os.environ.get("MIPIPE_BENCH_ATTEMPT_S", "0") or 0)
    wd = Watchdog(max(10.0, budget - 10.0) if budget > 0 else 600.0)
    rows = []
    out = {"P": None, "rows": rows, "complete": False}
    with wd.step():
        rank, world, local_rank, device = init_distributed()
        out["P"] = world
        _, _, B, S = (int(x) for x in a.ref_args.split(","))
        gpu = device.type == "cuda"
        p2p = P2P(None, list(range(world)), device) if (gpu and world > 1) else None
        grid = ref_grid(a, world)
    for gi, (L, H) in enumerate(grid):
        # every rank runs the same configs: rank 0 decides (time) and broadcasts
        go = torch.tensor([1.0 if (budget <= 0 or time.monotonic() - t_start < 0.8 * budget) else 0.0],
                          dtype=torch.float64, device=device)
        if world > 1:
            dist.broadcast(go, src=0)
        if float(go.item()) < 0.5:
            break
        steps, warmup = (a.steps, a.warmup) if gi == 0 else (5, 2)
        for sched in SCHEDULES:
            with wd.step():
                m = 4
                if sched != "Interleaved1F1B" and m < world:
                    m = world      # torch needs m >= stages for one stage per rank (schedules.py:578-583)
                torch.manual_seed(1234 + rank)
                args = ModelArgs(n_layers=L, n_heads=H)
                x = torch.randint(0, args.vocab_size, (B, S), dtype=torch.long, device=device)
                y = torch.randint(0, args.vocab_size, (B, S), dtype=torch.long, device=device)
                if gpu:
                    schedule = native_reference_schedule(args, sched, rank, world, B, S, m, device,
                                                         precision="fp32", p2p=p2p)
                    engine = "native fp32 kernels"
                else:
                    spw = stages_per_worker(sched, L, world)
                    stages = [manual_model_split(Transformer(args), rank + world * i, world * spw, device)
                              for i in range(spw)]
                    cls = get_schedule_class(sched)
                    schedule = cls(stages if spw > 1 or sched == "Interleaved1F1B" else stages[0], n_microbatches=m,
                                   loss_fn=tokenwise_loss_fn(args.vocab_size))
                    engine = "torch CPU (autograd)"
                if world > 1:
                    dist.barrier()
                met = run_train_iterations(schedule, x, y, rank, world, num_iterations=steps, warmup=warmup,
                                           device=device, measure_bubble=not a.no_bubble)
                el = torch.tensor([met["elapsed_time"]], dtype=torch.float64, device=device)
                if world > 1:
                    dist.all_reduce(el, op=dist.ReduceOp.MAX)
                rt = schedule.runtime
                last = torch.tensor([met["throughput"] if rank == world - 1 else 0.0], dtype=torch.float64,
                                    device=device)
                if world > 1:
                    dist.all_reduce(last, op=dist.ReduceOp.SUM)
                row = {"L": L, "H": H, "P": world, "schedule": sched, "v": rt.v, "microbatches": rt.m,
                       "tok_s": round(met["tokens_processed"] / float(el.item()), 1),
                       "tok_s_last_rank_timer": round(float(last.item()), 1),
                       "ms_per_step": round(float(el.item()) / steps * 1e3, 3), "steps": steps, "warmup": warmup,
                       "bubble_fraction": None if met.get("bubble_fraction") is None else
                       round(met["bubble_fraction"], 4),
                       "analytic_bubble": None if met.get("analytic_bubble") is None else
                       round(met["analytic_bubble"], 4),
                       "precision": met.get("precision", "fp32"), "engine": engine,
                       "native_runner": met.get("native_runner"), "lanes": met.get("lanes"), "p2p": rt.p2p.kind}
                nb = published(L, H, world, sched) if a.ref_args.split(",")[2:] == ["32", "128"] else None
                if nb:
                    row["nb_row"] = {"tok_s": nb, "P": world, "source": f"BASELINE.md Table 1 "
                                                                       f"(nb:{SOURCE_LINE[(L, H, world, sched)]}), "
                                                                       "10-core CPU"}
                    row["x_vs_nb"] = round(row["tok_s"] / nb, 1)
                rows.append(row)
                if rank == 0:
                    emit(out, partial=True)   # a budget kill still leaves the runs done so far
                del schedule, rt
                gc.collect()
                if gpu:
                    torch.cuda.empty_cache()
    out["complete"] = len(rows) == len(grid) * len(SCHEDULES)
    out["wall_s"] = round(time.monotonic() - t_start, 1)
    if rank == 0:
        emit(out)
    with wd.step():
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
    if n != world_env and world_env > 1 and not (a.phase == "ref" and a.ref_p == world_env):
        # (a reference child on ranks 0..P-1 of the launch runs with WORLD_SIZE = P)
        raise SystemExit(f"--gpus {n} but WORLD_SIZE={world_env}")
    if os.environ.get("MIPIPE_BENCH_CHILD") != "1" and not a.no_supervise and a.phase == "sched":
        # (an explicit internal --phase runs that phase here, e.g. under a profiler)
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
    if a.phase == "ref":
        run_ref(a)
    elif a.phase == "plan":
        run_plan(a)
    elif a.phase == "rate":
        run_rate(a)
    else:
        run(a)


if __name__ == "__main__":
    main()
