"""bench.py hang safety on CPU/gloo (2 ranks, tiny GPT-2): a rank that stops answering
must end the run non-zero with the program grid printed (watchdog), and a stall confined
to the first attempt must be retried by the supervisor into a valid JSON line
(the reference's launcher joins with no timeout, nb:324-325)."""
import json
import os
import subprocess
import sys

import pytest

from dist_utils import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--model", "gpt2-tiny", "--vocab", "256", "--mbs", "1", "--seq", "32", "--steps", "3", "--warmup", "1",
        "--step-timeout", "4"]


def _bench(extra, stall, timeout=240, **envx):
    env = dict(os.environ, MIPIPE_FAULT_STALL=stall, OMP_NUM_THREADS="1", MIPIPE_BENCH_ATTEMPT_S="90")
    env.update(envx)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py")] + ARGS + extra
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd="/tmp")


def test_stalled_rank_exits_nonzero_with_grid():
    r = _bench(["--max-attempts", "1"], "1:2")
    assert r.returncode != 0
    assert "[mipipe watchdog]" in r.stderr
    assert "Rank 0" in r.stderr and "Rank 1" in r.stderr and "Step 00:" in r.stderr   # the program grid
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_supervisor_retries_a_stalled_attempt():
    r = _bench([], "1:2:0")     # only attempt 0 stalls
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["attempt"] == 1 and out["n_gpus"] == 2 and out["value"] > 0
    assert out["config"]["parallelism"] == "pp2"
    assert "attempt 0" in r.stderr


def test_default_budget_fits_the_driver_timeout():
    """The attempt budgets of the defaults never add up past 560 s of the driver's 600 s,
    however long each attempt hangs (each runs out its whole budget)."""
    sys.path.insert(0, ROOT)
    import bench
    t, n = 0.0, 0
    while n < 10:
        b = bench.attempt_budget(t)
        if b <= 0:
            break
        t += b + 5.0        # the attempt hangs to its limit; killing it takes <= 5 s
        n += 1
    assert n >= 2 and t <= 560.0, (n, t)


def test_baseline_configs_are_planned_last_at_their_gpu_count():
    """BASELINE.json's named multi-GPU configs run after the headline, the other schedules
    and the reference's fp32 config, at the GPU count they name (4: GPT-2 small 1F1B m=8;
    8: GPT-2 medium interleaved, Llama-3 8B PP=8 and DP2 x PP4), and never by default off a
    GPU box."""
    sys.path.insert(0, ROOT)
    import bench
    old = os.environ.get("WORLD_SIZE")
    try:
        for world, n in ((4, 1), (8, 3), (2, 0)):
            os.environ["WORLD_SIZE"] = str(world)
            a = bench.parse(["--base-configs", "1", "--ref-fp32", "1"])
            ph = bench.plan_phases(a, ["--steps", "3"])
            kinds = [k for _, k, _, _ in ph]
            assert kinds.count("base") == n
            if n:
                assert kinds[-n:] == ["base"] * n and kinds.index("base") > max(i for i, k in enumerate(kinds)
                                                                                if k in ("ref", "sched"))
                argv = ph[-n][2]
                assert argv[:2] == ["--steps", "3"] and "--model" in argv
            a = bench.parse(["--ref-fp32", "0"])
            if not os.path.exists("/dev/kfd"):
                assert not [p for p in bench.plan_phases(a, []) if p[1] == "base"]
        os.environ["WORLD_SIZE"] = "8"
        assert any("llama3-8b" in x for x in bench.plan_phases(bench.parse(["--base-configs", "1"]), [])[-1][2])
    finally:
        if old is None:
            os.environ.pop("WORLD_SIZE", None)
        else:
            os.environ["WORLD_SIZE"] = old


def test_merge_results_baseline_configs_block():
    sys.path.insert(0, ROOT)
    import bench
    head = {"value": 10.0, "n_gpus": 4, "config": {"schedule": "1F1B"}}
    res = {"b0": {"value": 7.0, "ms_per_step": 3.0, "config": {"model": "gpt2-small", "schedule": "1F1B",
                                                               "microbatches": 8, "micro_batch": 16}}}
    out = bench.merge_results(head, res, bench.parse(["--ref-fp32", "0"]))
    (name, e), = out["baseline_configs"].items()
    assert "gpt2-small" in name and e["tok_s"] == 7.0 and e["microbatches"] == 8 and e["model"] == "gpt2-small"
    res = {"b0": {"skipped": "time"}}
    assert bench.merge_results(head, res, bench.parse([]))["baseline_configs"][name] == {"skipped": "time"}


def test_attempt_modes_and_last_resort_gloo():
    """The headline's attempts go from the full native path to ever more conservative ones;
    the last moves every process group to gloo (RCCL unusable on the node), so a number --
    labelled by attempt_mode / p2p -- still comes out."""
    sys.path.insert(0, ROOT)
    import bench
    modes = [m for m, _ in bench.ATTEMPTS]
    assert modes[0] == "auto" and modes[-1] == "gloo"
    base = {"TORCHELASTIC_USE_AGENT_STORE": "1", "PATH": "/usr/bin"}
    e = bench.child_env(base, "gloo", 4, 29600, 120.0, "/tmp/x.json")
    assert e["MIPIPE_DIST_BACKEND"] == "gloo" and e["MIPIPE_P2P"] == "auto" and e["MIPIPE_BENCH_MODE"] == "gloo"
    assert "TORCHELASTIC_USE_AGENT_STORE" not in e and e["MASTER_PORT"] == "29600"
    e = bench.child_env(base, "auto-safe", 1, 29601, 120.0, "/tmp/x.json")
    assert e["MIPIPE_P2P"] == "auto" and e["MIPIPE_COLL_OVERLAP"] == "0" and e["MIPIPE_PP_LANES"] == "0"
    assert e["MIPIPE_RECV_EARLY"] == "0"
    assert "MIPIPE_DIST_BACKEND" not in e
    e = bench.child_env(base, "torch", 2, 29602, 120.0, "/tmp/x.json")
    assert e["MIPIPE_P2P"] == "torch" and "MIPIPE_COLL_OVERLAP" not in e


def test_two_stalled_attempts_end_nonzero_within_the_deadline():
    """Every attempt stalls: the supervisor gives up non-zero inside its global deadline
    (scaled down here to 80 s; the default is 540 s, test above)."""
    import time
    t0 = time.monotonic()
    r = _bench([], "1:2", timeout=200, MIPIPE_BENCH_DEADLINE_S="80", MIPIPE_BENCH_ATTEMPT_S="40")
    dt = time.monotonic() - t0
    assert r.returncode != 0
    assert dt < 80 + 25, dt
    assert "attempt 0" in r.stderr and "attempt 1" in r.stderr and "giving up" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_eight_ranks_gpt2_small_layout():
    """The N = 8 launch the driver makes (bench.py --gpus 8 self-launch under
    torch.distributed.run, supervisor, PP = 8 over GPT-2 small's 12 layers with the
    distributed head, m = 4P = 32) completes on CPU/gloo and prints one valid line."""
    env = dict(os.environ, OMP_NUM_THREADS="1", MIPIPE_BENCH_ATTEMPT_S="200", MASTER_PORT=str(free_port()))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "1", "--mbs", "1",
           "--seq", "32", "--vocab", "512", "--base-configs", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    c = out["config"]
    assert out["n_gpus"] == 8 and out["value"] > 0 and c["parallelism"] == "pp8" and c["microbatches"] == 32
    assert c["model"] == "gpt2-small" and len(c["layer_split"]) == 8 * c["v"]
    assert sum(b - a for a, b in c["layer_split"]) == 12
    assert c["head"].startswith("distributed") and out["bubble_fraction"] is not None


def test_bench_default_batch_is_128_sequences_per_gpu():
    """Weak-scaling contract of bench.py's defaults: 128 sequences per GPU per step -- one
    GPU as 2 microbatches of 64, a pipeline of N as 4N microbatches of 32 (global 128 N)."""
    env = dict(os.environ, OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--model", "gpt2-tiny", "--vocab", "256", "--seq", "16",
           "--steps", "1", "--warmup", "1", "--no-bubble"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    c = out["config"]
    assert (c["micro_batch"], c["microbatches"], c["global_batch"]) == (64, 2, 128)
    assert out["scaling"] == "weak" and out["n_gpus"] == 1


def test_bench_pipeline_plans_the_microbatch_size():
    """No --mbs at PP > 1: rank 0's supervisor plans the microbatch size in a CPU-only child
    (engine.pick_microbatch), every rank's children run it, the batch stays 128 sequences
    per GPU, and the record carries the plan (config.mbs_choice)."""
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_PORT=str(free_port()))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "gpt2-tiny", "--vocab", "256",
           "--seq", "8", "--steps", "1", "--warmup", "1", "--no-bubble", "--schedules", "none"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    c = out["config"]
    plan = c["mbs_choice"]
    assert plan["mbs"] in (16, 32) and set(plan["scores"]) == {"16", "32"}, plan
    assert c["micro_batch"] == plan["mbs"] and c["microbatches"] == plan["microbatches"]
    assert c["micro_batch"] * c["microbatches"] == 256 and c["global_batch"] == 256


def test_bench_four_ranks_measures_all_three_schedules():
    """One ``bench.py --gpus 4`` call (CPU/gloo) measures the reference's comparison --
    GPipe, 1F1B and Interleaved1F1B on the same model/config, each with its measured and
    analytic bubble -- and the record carries the transport's bytes per step."""
    import time
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_PORT=str(free_port()))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--base-configs", "0",
           "--compare-model", "same"] + ARGS[:-2]
    t0 = time.monotonic()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd="/tmp")
    dt = time.monotonic() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    sch = out["schedules"]
    # entries are labelled by what they ran ("<schedule>+lag<k>" with a head lag);
    # "1F1B" is the reference's warmup depth (head lag capped at 0)
    by = {}
    for name, e in sch.items():
        by.setdefault(e["schedule"], []).append(name)
        assert name.split(" ")[0] == e["schedule"] + (f"+lag{e['head_lag']}" if e["head_lag"] else ""), (name, e)
    assert set(by) == {"GPipe", "1F1B", "Interleaved1F1B", "ZBH1"}, sch
    assert sch["1F1B"]["head_lag"] == 0
    for name, e in sch.items():
        assert e["tok_s"] > 0 and e["bubble_fraction"] is not None and e["analytic_bubble"] is not None, (name, e)
        assert e["p2p_bytes_per_step"] > 0 and len(e["stash_slots_per_rank"]) == 4
    il = sch[by["Interleaved1F1B"][0]]
    gp = sch[by["GPipe"][0]]
    # 4 layers over 4 ranks: two chunks per rank would leave virtual stages empty, so
    # interleaved falls back to one chunk -- the reference's own rule when L % 2P != 0
    # (helper:181-183; VERDICT r4: no empty range in any layer split)
    assert il["v"] == 1 and gp["v"] == 1
    assert il["analytic_bubble"] == sch["1F1B"]["analytic_bubble"]
    for name, e in sch.items():
        assert all(b > a for a, b in e["layer_split"]), (name, e["layer_split"])
    assert gp["speedup_vs_gpipe"] == 1.0
    # --schedule auto: the headline is the best-planned schedule, and it is measured once
    head = out["config"]["schedule"]
    hl = head + (f"+lag{out['config']['head_lag']}" if out["config"]["head_lag"] else "")
    assert out["value"] == sch[hl]["tok_s"] and set(out["config"]["schedule_choice"]["auto"]) == set(by)
    plans = out["config"]["schedule_choice"]["plans"]
    assert all({"head_lag", "stash_slots_max", "planned_gb_max"} <= set(p) for p in plans.values()), plans
    eff = out["config"]["schedule_choice"]["auto"]
    # the best plan among candidates that beat 1F1B by their margin (3 % with more p2p
    # than 1F1B -- interleaved v > 1 --, 1 % with the same messages), else 1F1B
    v_of = {s: sch[names[0]]["v"] for s, names in by.items()}
    beats = [k for k in eff if k != "1F1B" and eff[k] >= eff["1F1B"] * (1.03 if v_of.get(k, 1) > 1 else 1.01)]
    assert head == (max(beats, key=lambda k: eff[k]) if beats else "1F1B"), (head, eff, v_of)
    assert out["p2p_bytes_per_step"] > 0 and "rccl_ranks" in out
    # every rank's live concurrency features (VERDICT r4 #6c): one entry per rank
    conc = out["per_rank_concurrency"]
    assert len(conc) == 4 and all(set(c) >= {"queue_probe", "rccl_communicators", "lanes", "p2p_channels",
                                             "collective_placement", "comm_audit"} for c in conc), conc
    assert all(str(c["comm_audit"]).startswith("ok (") for c in conc), conc
    assert dt < 540, dt


def test_extra_phases_never_push_past_the_deadline():
    """Worst case of the supervisor's plan: the headline succeeds late, then every other
    schedule and reference child hangs until it is killed at its budget -- the run still
    ends inside 560 s of the driver's 600 s."""
    sys.path.insert(0, ROOT)
    import bench
    for head_wall in (20.0, 60.0, 150.0, 230.0):
        t = head_wall + 1.0                 # headline attempt 0 succeeded
        ref_wall = None
        # N = 8: four other schedules, then the reference grid at P = 2, 4 (27 runs each) and 8
        for kind in ["sched"] * 4 + ["ref:27", "ref:27", "ref:3"]:
            b, est = bench.extra_budget(kind, bench.DEADLINE_S - t, bench.ATTEMPT_CAP_S, head_wall, ref_wall)
            if b <= 0:
                continue
            assert b <= bench.DEADLINE_S - t - 10.0
            t += b + 5.0                    # hangs to its limit; the kill takes <= 5 s
            if kind.startswith("ref"):
                ref_wall = (b * 1.25 + 5) / int(kind.split(":")[1])
        assert t <= 560.0, (head_wall, t)


def test_merge_results_reference_block_and_speedups():
    """bench.merge_results: the headline line + every schedule (the headline's own included)
    with speedup vs GPipe, and the reference fp32 rows, each next to the published row of the
    SAME (L, H, P, schedule) -- P = 2 / 4 only; P = 1 and P = 8 rows carry none (VERDICT r4:
    never P = 8 against the P = 2 row)."""
    sys.path.insert(0, ROOT)
    import argparse
    import bench
    head = {"value": 100.0, "n_gpus": 8, "ms_per_step": 10.0, "bubble_fraction": 0.0, "analytic_bubble": 0.0,
            "config": {"schedule": "1F1B", "v": 1, "microbatches": 2}}

    def row(L, H, P, s, t):
        from mipipe.bench.published import published, SOURCE_LINE
        r = {"L": L, "H": H, "P": P, "schedule": s, "tok_s": t}
        nb = published(L, H, P, s)
        if nb:
            r["nb_row"] = {"tok_s": nb, "P": P, "source": f"nb:{SOURCE_LINE[(L, H, P, s)]}"}
            r["x_vs_nb"] = round(t / nb, 1)
        return r
    res = {"x_GPipe": {"value": 80.0, "config": {"schedule": "GPipe", "v": 1}},
           "x_Interleaved1F1B": {"error": "child exited rc=17 without a result after 50s"},
           "r2": {"P": 2, "complete": True, "rows": [row(8, 8, 2, "GPipe", 167132.0), row(8, 8, 2, "1F1B", 164953.0),
                                                     row(8, 8, 2, "Interleaved1F1B", 179630.0)]},
           "r4": {"P": 4, "complete": False, "rows": [row(8, 8, 4, "GPipe", 167515.0)]},
           "r8": {"P": 8, "complete": True, "rows": [row(8, 8, 8, "GPipe", 100.0), row(8, 8, 8, "1F1B", 120.0)]}}
    a = argparse.Namespace(ref_args="8,8,32,128")
    out = bench.merge_results(head, res, a)
    s = out["schedules"]
    assert s["1F1B"]["tok_s"] == 100.0 and s["GPipe"]["speedup_vs_gpipe"] == 1.0
    assert s["1F1B"]["speedup_vs_gpipe"] == 1.25 and "error" in s["Interleaved1F1B"]
    r = out["reference_fp32"]
    for x in r["rows"]:
        assert "nb_row" not in x or x["nb_row"]["P"] == x["P"], x
        assert ("nb_row" in x) == (x["P"] in (2, 4)), x
    p2 = {x["schedule"]: x for x in r["rows"] if x["P"] == 2}
    assert p2["GPipe"]["x_vs_nb"] == 100.0 and p2["1F1B"]["speedup_vs_gpipe"] == round(164953 / 167132, 4)
    assert r["summary"]["P2"]["published_rows"] == 3 and r["summary"]["P8"]["published_rows"] == 0
    assert r["status"]["P4"]["complete"] is False and r["status"]["P2"]["configs"] == 1
    # per_schedule: L8 H8 at P = N (8)
    assert set(r["per_schedule"]) == {"GPipe", "1F1B"} and r["tok_s"] == 120.0
    res["r2"] = {"skipped": "time"}
    assert bench.merge_results(head, res, a)["reference_fp32"]["status"]["P2"] == {"skipped": "time"}


def test_bench_eight_ranks_reference_at_published_pipeline_sizes():
    """an N = 8 call runs the reference's fp32 config at P = 2 and P = 4 on rank
    subsets (ranks 0..P-1) as well as at P = 8, and every row's published comparison is the
    row of the same P (here L4 H4, the cheapest published config, on CPU/gloo)."""
    env = dict(os.environ, OMP_NUM_THREADS="1", MIPIPE_BENCH_ATTEMPT_S="240", MASTER_PORT=str(free_port()),
               MIPIPE_BENCH_REF_RUN_S="40")    # a d768 model on one CPU thread per rank
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "1", "--mbs",
           "1", "--seq", "32", "--vocab", "512", "--model", "gpt2-tiny", "--base-configs", "0", "--schedules", "none",
           "--ref-fp32", "1", "--ref-grid", "4,4", "--no-bubble"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=540, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    ref = out["reference_fp32"]
    assert set(ref["status"]) == {"P2", "P4", "P8"}, ref["status"]
    by_p = {}
    for x in ref["rows"]:
        by_p.setdefault(x["P"], set()).add(x["schedule"])
        assert (x["L"], x["H"]) == (4, 4) and x["tok_s"] > 0
        if x["P"] in (2, 4):
            assert x["nb_row"]["P"] == x["P"] and x["x_vs_nb"] > 0, x
        else:
            assert "nb_row" not in x
    assert by_p == {P: {"GPipe", "1F1B", "Interleaved1F1B"} for P in (2, 4, 8)}, by_p


def test_bench_eight_ranks_compares_the_schedules_it_names():
    """at N = 8 the schedule comparison runs on a model that interleaves at
    P = 8 (here gpt2-tiny with 16 layers, CPU/gloo; on the GPU box GPT-2 medium), the
    Interleaved1F1B entry really runs v = 2, a "1F1B" entry runs the reference's warmup
    depth (per-rank stash slots <= P - r + lanes - 1), the planner's deeper 1F1B is labelled
    with its lag, and every entry reports its head lag and per-rank stash slots."""
    env = dict(os.environ, OMP_NUM_THREADS="1", MIPIPE_BENCH_ATTEMPT_S="240", MASTER_PORT=str(free_port()))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "1", "--mbs", "1",
           "--seq", "32", "--vocab", "512", "--model", "gpt2-tiny", "--compare-model", "gpt2-tiny:16",
           "--base-configs", "0", "--ref-fp32", "0", "--no-bubble"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=540, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["schedules_model"] == "gpt2-tiny:16" and "schedules_note" in out
    sch = out["schedules"]
    P = 8
    for name, e in sch.items():
        assert e["model"] == "gpt2-tiny:16" and e["microbatches"] == 32 and e["micro_batch"] == 1, (name, e)
        assert "head_lag" in e and len(e["stash_slots_per_rank"]) == P, (name, e)
    il = [e for e in sch.values() if e["schedule"] == "Interleaved1F1B"]
    assert il and il[0]["v"] == 2, sch
    ref = sch["1F1B"]
    assert ref["head_lag"] == 0 and ref["v"] == 1
    lanes = max(c["lanes"] for c in out["per_rank_concurrency"])
    for rank, slots in enumerate(ref["stash_slots_per_rank"]):
        assert sum(slots.values()) <= P - rank + lanes - 1, (rank, slots)
    # the planned 1F1B ran too, labelled by its lag (or, if the planner chose lag 0, as a
    # second "1F1B" entry)
    planned = [k for k, e in sch.items() if e["schedule"] == "1F1B" and k != "1F1B"]
    assert planned and all(k.startswith("1F1B+lag") or k.startswith("1F1B (planned)") for k in planned), sch
    assert {"GPipe", "ZBH1"} <= {e["schedule"] for e in sch.values()}
