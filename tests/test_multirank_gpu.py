"""The full multi-process pipeline stack on the GPU: 2 and 4 ranks sharing one device
(gloo carries the traffic through host memory, MIPIPE_DIST_BACKEND=gloo) must train
exactly like one process -- HIP kernels, distributed head, schedules and HIP graphs in
the real multi-rank runtime.  RCCL itself needs one GPU per rank and is exercised by
the 8-GPU scaling bench."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, *args, port, backend="gloo", extra_env=None):
    env = dict(os.environ, MIPIPE_DIST_BACKEND=backend, OMP_NUM_THREADS="2", **(extra_env or {}))
    if backend != "gloo":
        env.pop("MIPIPE_DIST_BACKEND")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tools", "mp_gpu_check.py")] + list(args)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


@pytest.fixture(scope="module")
def reference():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return _run(1, port=29771)["losses"]


@pytest.fixture(scope="module")
def reference8():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return _run(1, "--layers", "8", port=29761)["losses"]


@pytest.mark.parametrize("n,schedule,graphs,split,dp", [(2, "1F1B", 0, 1, 1), (2, "ZBH1", 1, 1, 1),
                                                        (4, "ZBH1", 1, 1, 1),
                                                        (4, "1F1B", 1, 1, 1), (4, "GPipe", 0, 0, 1),
                                                        (2, "ZBV", 0, 1, 1), (4, "1F1B", 1, 1, 2),
                                                        (2, "1F1B", 1, 1, 2)])
def test_multirank_gpu_matches_single(reference, n, schedule, graphs, split, dp):
    """dp=2: DP x PP (2 x 2) with HIP graphs -- the stages' DP all-reduce replays as a
    recorded CALL on the native runner's tape.  (2, dp=2) is DP2 x PP1: microbatch lanes
    on each replica, joined (lane gradients summed) before the DP all-reduce."""
    res = _run(n, "--schedule", schedule, "--graphs", str(graphs), "--split-head", str(split), "--dp", str(dp),
               port=29772 + n + 10 * graphs + 20 * split + 40 * dp)
    # bf16 kernels + split-K atomics: equal up to reduction-order rounding
    assert res["losses"] == pytest.approx(reference, rel=2e-3)
    # with graphs, steps after the first replay run from the native stage runner's tape
    # (gloo transfers recorded as CALLs)
    assert res["native_runner"] == bool(graphs), res["native_reason"]
    # microbatch lanes at PP > 1 too (one stage per rank, graphs): two lane streams with
    # per-lane stage + head gradients, sends ordered after their lane
    if graphs and schedule in ("1F1B", "GPipe"):
        assert res["lanes"] >= 2, res


@pytest.fixture(scope="module")
def reference_5steps():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return _run(1, "--steps", "5", port=29769)["losses"]


@pytest.mark.parametrize("split,env", [(0, {}), (1, {"MIPIPE_HEAD_ZERO": "0"})])
def test_multirank_gpu_replayed_steps_reduce_once(reference_5steps, split, env):
    """steps replayed from the native tape must not repeat per-step work the
    runtime issues itself.  split=0: GPT-2's tied embedding lives on the first and the last
    stage and its two gradients are summed once per step (post_step, outside the tape; it
    was also recorded, so every replayed step summed it twice).  split=1 with a replicated
    head (MIPIPE_HEAD_ZERO=0): the head gradient is all-reduced over the pipeline after the
    lane merge, so the clip norm must come from the reduced gradient, not the merge's
    sum of squares.  Five steps: two replayed after the capture and the recording step."""
    res = _run(2, "--schedule", "1F1B", "--graphs", "1", "--split-head", str(split), "--steps", "5",
               port=29930 + split, extra_env=env)
    assert res["native_runner"], res["native_reason"]
    assert res["lanes"] >= 2, res
    assert res["losses"] == pytest.approx(reference_5steps, rel=2e-3)


@pytest.mark.parametrize("n,graphs,split", [(2, 1, 1), (4, 1, 1), (4, 0, 0)])
def test_multirank_gpu_interleaved_matches_single(reference8, n, graphs, split):
    """Interleaved 1F1B with 2 virtual stages per rank (BASELINE config 3's schedule;
    reference helper:182-185, 204-211): 8 layers over 2*PP stages, HIP graphs + native
    tape, with and without the distributed head, vs one process."""
    res = _run(n, "--schedule", "Interleaved1F1B", "--vstages", "2", "--layers", "8", "--graphs", str(graphs),
               "--split-head", str(split), port=29860 + n + 10 * graphs + 20 * split)
    assert res["losses"] == pytest.approx(reference8, rel=2e-3)
    assert res["native_runner"] == bool(graphs), res["native_reason"]
    if graphs:   # two lanes with two stages per rank: each stage merged at its own REDUCE_GRAD
        assert res["lanes"] == 2, res


@pytest.mark.parametrize("n,schedule,graphs,split,dp", [(2, "1F1B", 1, 1, 1), (4, "1F1B", 1, 1, 1),
                                                        (4, "GPipe", 0, 0, 1), (8, "1F1B", 1, 1, 2)])
def test_rccl_one_gpu_per_rank_matches_single(reference, n, schedule, graphs, split, dp):
    """The real multi-GPU path: one rank per GPU, RCCL (nccl backend) with the native p2p
    engine, HIP graphs + the native tape.  Needs n GPUs in one node (skipped on the
    one-GPU box: two RCCL ranks cannot share a device, tools/rccl_shared_gpu_probe.py)."""
    if torch.cuda.device_count() < n:
        pytest.skip(f"needs {n} GPUs")
    res = _run(n, "--schedule", schedule, "--graphs", str(graphs), "--split-head", str(split), "--dp", str(dp),
               port=29850 + n + 10 * graphs + 20 * split + 40 * dp, backend="nccl")
    assert res["losses"] == pytest.approx(reference, rel=2e-3)
    assert res["p2p"] == "native", res
    assert res["native_runner"] == bool(graphs), res["native_reason"]


@pytest.mark.parametrize("schedule,v", [("1F1B", 1), ("ZBH1", 1)])
def test_rccl_pp8_matches_single(reference8, schedule, v):
    """PP = 8 over 8 GPUs (one layer per stage), RCCL + native p2p + graphs.  Skipped
    below 8 GPUs."""
    if torch.cuda.device_count() < 8:
        pytest.skip("needs 8 GPUs")
    args = ["--layers", "8", "--schedule", schedule, "--graphs", "1", "--split-head", "1"]
    if v > 1:
        args += ["--vstages", str(v)]
    res = _run(8, *args, port=29890 + v, backend="nccl")
    assert res["losses"] == pytest.approx(reference8, rel=2e-3)
    assert res["p2p"] == "native", res


def test_multirank_stash_follows_the_schedule():
    """with HIP graphs on every rank (4 ranks, P = 4, m = 16), each rank holds
    its schedule's in-flight activation stashes: 1F1B P - r per microbatch lane (rounded),
    GPipe all 16 -- the HBM above each rank's post-init level is ordered GPipe > 1F1B on
    every rank, and on the last rank (1F1B: one stash per lane) well under half of GPipe's.
    The head lag is capped at 0: this toy model is all p2p latency in the cost model, so the
    head planner would otherwise buy a lag of m (= GPipe's stash) for a 4x shorter plan."""
    res = {}
    for sched in ("GPipe", "1F1B"):
        res[sched] = _run(4, "--schedule", sched, "--graphs", "1", "--split-head", "1", "--microbatches", "16", "--mem", "1",
                          "--steps", "2", port=29940 + len(sched), extra_env={"MIPIPE_HEAD_MAX_LAG": "0"})
    g, o = res["GPipe"]["mem"], res["1F1B"]["mem"]
    lanes = res["1F1B"]["lanes"]
    assert g["stash_slots"] == [16] * 4, g
    assert all(s_ <= -(-(4 - r) // lanes) * lanes for r, s_ in enumerate(o["stash_slots"])), (o, lanes)
    for r in range(4):
        assert o["peak_above_init"][r] < g["peak_above_init"][r], (r, o, g)
    assert o["peak_above_init"][3] < 0.5 * g["peak_above_init"][3], (o, g)


@pytest.mark.parametrize("split_head,extra", [(0, {}), (1, {"MIPIPE_HEAD_ZERO": "0"})])
def test_multirank_lanes_keep_the_clip_norm(split_head, extra):
    """with microbatch lanes the fused lane merge's sum of squares must
    not stand in for the clip norm of an arena that is reduced further after the merge (the
    stage-0 arena holding a tied embedding; the replicated head with MIPIPE_HEAD_ZERO=0).
    PP = 2 with graphs: the pre-clip global norms of 4 steps with 2 lanes match one lane."""
    res = {}
    for lanes in ("2", "1"):
        res[lanes] = _run(2, "--graphs", "1", "--split-head", str(split_head), "--steps", "4", "--clip", "0.05",
                          port=29960 + 2 * split_head + int(lanes), extra_env={"MIPIPE_LANES": lanes, **extra})
    assert res["2"]["lanes"] == 2 and res["1"]["lanes"] == 1, (res["2"]["lanes"], res["1"]["lanes"])
    # (without the fix the first step's norm is 2 % off: the tied / replicated part counted unreduced)
    assert res["2"]["norms"] == pytest.approx(res["1"]["norms"], rel=5e-3), (res["2"]["norms"], res["1"]["norms"])
    assert res["2"]["losses"] == pytest.approx(res["1"]["losses"], rel=2e-3)


def test_multirank_stash_ring_zbh1_and_interleaved_train_like_gpipe():
    """The stash ring with split backwards (ZBH1: a stash's last reader is W) and with two
    virtual stages per rank (interleaved, v = 2, 8 layers): the same losses as GPipe over 3
    steps (HIP graphs, 4 ranks, m = 16), fewer slots than GPipe's 16 per stage on every rank
    and a lower HBM peak on the last rank."""
    res = {}
    for sched, extra in (("GPipe", ()), ("ZBH1", ()), ("Interleaved1F1B", ("--vstages", "2"))):
        res[sched] = _run(4, "--schedule", sched, "--layers", "8", "--graphs", "1", "--split-head", "1",
                          "--microbatches", "16", "--mem", "1", "--steps", "3", *extra,
                          port=29980 + len(sched), extra_env={"MIPIPE_HEAD_MAX_LAG": "0"})
    g = res["GPipe"]
    for sched in ("ZBH1", "Interleaved1F1B"):
        r = res[sched]
        assert r["losses"] == pytest.approx(g["losses"], rel=2e-3), (sched, r["losses"], g["losses"])
        nst = 2 if sched == "Interleaved1F1B" else 1
        assert all(s_ < 16 * nst for s_ in r["mem"]["stash_slots"]), (sched, r["mem"])
        assert r["mem"]["peak_above_init"][3] < g["mem"]["peak_above_init"][3], (sched, r["mem"], g["mem"])
