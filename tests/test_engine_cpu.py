"""End-to-end engine on CPU/gloo: a PP=2 (and PP=2 x DP=2) training step of a native
GPT-2 / Llama must produce the same loss and updated weights as PP=1."""
import pytest
import torch

import mipipe  # noqa: F401
from mipipe.engine import PipelineTrainer
from mipipe.models.config import NativeConfig

from dist_utils import run_world

CFG = dict(gpt2=lambda: NativeConfig.gpt2("tiny", vocab_size=100, d_model=64, n_layers=4, n_heads=4, d_ff=128,
                                          max_seq_len=16),
           llama=lambda: NativeConfig.llama3("tiny", vocab_size=100, d_model=64, n_layers=4, n_heads=4, n_kv_heads=2,
                                             d_ff=128, max_seq_len=16),
           gpt2_8=lambda: NativeConfig.gpt2("tiny", vocab_size=100, d_model=64, n_layers=8, n_heads=4, d_ff=128,
                                            max_seq_len=16),
           llama_8=lambda: NativeConfig.llama3("tiny", vocab_size=100, d_model=64, n_layers=8, n_heads=4,
                                               n_kv_heads=2, d_ff=128, max_seq_len=16))
M, MBS, S = 4, 2, 16


def _data(cfg, dp_rank=0, step=0):
    g = torch.Generator().manual_seed(7 + dp_rank + 100 * step)
    return (torch.randint(0, cfg.vocab_size, (M * MBS, S), generator=g),
            torch.randint(0, cfg.vocab_size, (M * MBS, S), generator=g))


def _train(name, pp, dp, schedule, steps=2, split_head=None, layer_ranges="auto", max_grad_norm=1.0,
           concat_dp=1, adam_eps=1e-8, lr=1e-3, v=None):
    """concat_dp=k (PP=1, DP=1 only): train on the concatenation of k DP replicas' batches
    (k*M microbatches) -- the single-process oracle of a DP=k run."""
    cfg = CFG[name]()
    if layer_ranges == "auto":
        layer_ranges = [(0, 2), (2, 4)] if (pp == 2 and not v) else None
    tr = PipelineTrainer(cfg, pp=pp, dp=dp, schedule=schedule, n_microbatches=M * concat_dp, mbs=MBS, seq_len=S, v=v,
                         device=torch.device("cpu"), dtype=torch.float32, lr=lr,
                         layer_ranges=layer_ranges, split_head=split_head, head_align=8,
                         max_grad_norm=max_grad_norm, adam_eps=adam_eps)
    losses = []
    for step in range(steps):
        if concat_dp > 1:
            parts = [_data(cfg, d, step) for d in range(concat_dp)]
            x, y = torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts])
        else:
            x, y = _data(cfg, tr.mesh.dp_rank, step)
        l = tr.train_step(x, y)
        if l is not None:
            losses.append(float(l))
    sd = {k: v.numpy().copy() for k, v in tr.state_dict().items()}
    return dict(losses=losses, sd=sd, audit=tr.comm_audit)


def _worker(rank, world, name, pp, dp, schedule, split_head=None, layer_ranges="auto", max_grad_norm=1.0,
            adam_eps=1e-8, lr=1e-3, v=None):
    return _train(name, pp, dp, schedule, split_head=split_head, layer_ranges=layer_ranges,
                  max_grad_norm=max_grad_norm, adam_eps=adam_eps, lr=lr, v=v)


@pytest.mark.parametrize("name", ["gpt2_8", "llama_8"])
@pytest.mark.parametrize("pp", [2, 4])
@pytest.mark.parametrize("split_head", [False, True])
def test_interleaved_v2_matches_pp1(name, pp, split_head):
    """Interleaved 1F1B with 2 virtual stages per rank (reference helper:182-185,
    204-211, 219-220; BASELINE config 3) on the native engine: PP=2 (4 stages) and PP=4
    (8 stages, loop placement: rank r holds stages r and r+P, wrap-around P-1 -> 0)."""
    ref = _train(name, 1, 1, "1F1B")
    res = run_world(_worker, pp, name, pp, 1, "Interleaved1F1B", split_head, None, 1.0, 1e-8, 1e-3, 2)
    holders = range(pp) if split_head else [pp - 1]      # loss lives on the last stage's rank
    for r in holders:
        assert res[r]["losses"] == pytest.approx(ref["losses"], rel=1e-5)
    for r in res.values():
        for k, w in r["sd"].items():
            torch.testing.assert_close(torch.from_numpy(w), torch.from_numpy(ref["sd"][k]), atol=1e-4, rtol=1e-4,
                                       msg=lambda m: f"{k}: {m}")


@pytest.mark.parametrize("name,split_head", [("gpt2", True), ("gpt2", False), ("llama", True)])
def test_dp2_pp2_matches_pp1_on_concatenated_batch_with_clipping(name, split_head):
    """DP=2 x PP=2 must equal one process training on both replicas' batches, with the
    grad-norm clip active (max_grad_norm 0.05): pins the 1/dp gradient scale of every
    arena -- including the replicated distributed head, all-reduced over pipeline x DP --
    and a tied embedding counted once in the global norm.  Adam eps = 1, lr = 1 makes the
    update ~ the clipped gradient itself (Adam is otherwise blind to a gradient's scale)."""
    ref = _train(name, 1, 1, "1F1B", max_grad_norm=0.05, concat_dp=2, adam_eps=1.0, lr=1.0)
    res = run_world(_worker, 4, name, 2, 2, "1F1B", split_head, "auto", 0.05, 1.0, 1.0)
    last = 1  # pipeline rank 1 of replica 0 holds the loss (every rank with a split head)
    # per-replica losses average to the concatenated-batch loss
    l0, l1 = res[last]["losses"], res[2 + last]["losses"]
    assert [(a + b) / 2 for a, b in zip(l0, l1)] == pytest.approx(ref["losses"], rel=1e-5)
    for r in res.values():
        for k, v in r["sd"].items():
            torch.testing.assert_close(torch.from_numpy(v), torch.from_numpy(ref["sd"][k]), atol=1e-4, rtol=1e-4,
                                       msg=lambda m: f"{k}: {m}")


@pytest.mark.parametrize("name", ["gpt2", "llama"])
def test_pp2_matches_pp1_with_active_clipping(name):
    """Clip active (0.05): the tied embedding's two copies (first and last stage) must
    count once in the global grad norm (Adam eps = 1, lr = 1: scale-sensitive updates)."""
    ref = _train(name, 1, 1, "1F1B", max_grad_norm=0.05, adam_eps=1.0, lr=1.0)
    res = run_world(_worker, 2, name, 2, 1, "1F1B", False, "auto", 0.05, 1.0, 1.0)
    assert res[1]["losses"] == pytest.approx(ref["losses"], rel=1e-5)
    for r in res.values():
        for k, v in r["sd"].items():
            torch.testing.assert_close(torch.from_numpy(v), torch.from_numpy(ref["sd"][k]), atol=1e-4, rtol=1e-4,
                                       msg=lambda m: f"{k}: {m}")


@pytest.mark.parametrize("name", ["gpt2", "llama"])
@pytest.mark.parametrize("schedule", ["1F1B", "GPipe", "ZBH1"])
@pytest.mark.parametrize("split_head", [False, True])
def test_pp2_matches_pp1(name, schedule, split_head):
    ref = _train(name, 1, 1, "1F1B")
    res = run_world(_worker, 2, name, 2, 1, schedule, split_head)
    assert res[1]["losses"] == pytest.approx(ref["losses"], rel=1e-5)
    if split_head:  # every rank reports the loss
        assert res[0]["losses"] == pytest.approx(ref["losses"], rel=1e-5)
    for r in res.values():
        for k, v in r["sd"].items():
            torch.testing.assert_close(torch.from_numpy(v), torch.from_numpy(ref["sd"][k]), atol=1e-4, rtol=1e-4,  # Adam amplifies fp32 reduction-order noise
                                       msg=lambda m: f"{k}: {m}")


def test_dp2_pp2_runs_and_replicas_agree():
    res = run_world(_worker, 4, "gpt2", 2, 2, "1F1B")
    # DP replicas of the same stage hold identical weights after the all-reduced update
    for a, b in [(0, 2), (1, 3)]:
        for k, v in res[a]["sd"].items():
            torch.testing.assert_close(torch.from_numpy(v), torch.from_numpy(res[b]["sd"][k]), atol=0, rtol=0)
    assert all(l == l for l in res[1]["losses"])


@pytest.mark.parametrize("schedule,layer_ranges", [("1F1B", None), ("GPipe", [(0, 1), (1, 2), (2, 3), (3, 4)]),
                                                   ("ZBH1", None)])
def test_pp4_distributed_head_matches_pp1(schedule, layer_ranges):
    """Distributed head over 4 ranks (uneven token chunks): same loss/weights as PP=1."""
    ref = _train("gpt2", 1, 1, "1F1B")
    res = run_world(_worker, 4, "gpt2", 4, 1, schedule, True, layer_ranges)
    for r in range(4):
        assert res[r]["losses"] == pytest.approx(ref["losses"], rel=1e-5)
    for r in res.values():
        for k, v in r["sd"].items():
            torch.testing.assert_close(torch.from_numpy(v), torch.from_numpy(ref["sd"][k]), atol=1e-4, rtol=1e-4,
                                       msg=lambda m: f"{k}: {m}")


def test_dp2_pp2_distributed_head_replicas_agree():
    res = run_world(_worker, 4, "llama", 2, 2, "1F1B", True)
    for a, b in [(0, 2), (1, 3), (0, 1)]:
        for k, v in res[a]["sd"].items():
            if k in res[b]["sd"]:
                torch.testing.assert_close(torch.from_numpy(v), torch.from_numpy(res[b]["sd"][k]), atol=0, rtol=0)


@pytest.mark.parametrize("split_head", [False, True])
def test_pp2_zbv_matches_pp1(split_head):
    ref = _train("gpt2", 1, 1, "1F1B")
    res = run_world(_worker, 2, "gpt2", 2, 1, "ZBV", split_head, None)
    # V placement: the last stage (and the loss) lives on rank 0
    assert res[0]["losses"] == pytest.approx(ref["losses"], rel=1e-5)
    for r in res.values():
        for k, v in r["sd"].items():
            torch.testing.assert_close(torch.from_numpy(v), torch.from_numpy(ref["sd"][k]), atol=1e-4, rtol=1e-4,
                                       msg=lambda m: f"{k}: {m}")


def test_recompute_auto_plan():
    """recompute="auto": the HBM plan keeps the whole stash when it fits (Llama-3 8B at
    seq 8192 on one 288 GB MI355X, PP=1: ~203 GB planned, 186 GB measured) and recomputes
    when it does not (a hypothetical 64 GB device)."""
    import torch
    from mipipe.engine import max_inflight_microbatches, plan_recompute
    from mipipe.models.config import NativeConfig
    from mipipe.models.native import balanced_layer_ranges
    from mipipe.parallel.schedules import generate
    import mipipe.engine as E

    cfg = NativeConfig.llama3("8b")
    lr = balanced_layer_ranges(cfg, 1, 8192, head_on_last=True)
    order = generate("1F1B", 1, 2, 1, "loop")[0]
    assert max_inflight_microbatches(order, {0}) == 1
    orig = E.torch.cuda.get_device_properties
    try:
        for gb, want in ((288, False), (64, True)):
            E.torch.cuda.get_device_properties = lambda d, gb=gb: type("P", (), {"total_memory": gb * 2 ** 30})()
            plan = plan_recompute(cfg, lr, [0], order, 1, 8192, torch.device("cuda", 0), head_tokens=8192)
            assert plan["recompute"] is want, plan
        assert 180e9 < plan["bytes_no_recompute"] < 230e9
        # distributed head, Llama-3 8B PP=8: ZeRO-1 keeps 1/8 of the head's master + Adam
        # moments per rank (the bf16 weights, W^T copy and f32 gradient stay whole)
        l8 = balanced_layer_ranges(cfg, 8, 8192, head_on_last=False)
        o8 = generate("1F1B", 8, 16, 1, "loop")[7]
        full = plan_recompute(cfg, l8, [7], o8, 1, 8192, torch.device("cuda", 0), head_tokens=1024)
        zero = plan_recompute(cfg, l8, [7], o8, 1, 8192, torch.device("cuda", 0), head_tokens=1024, head_shards=8)
        assert zero["head_optimizer_bytes"] <= full["head_optimizer_bytes"] / 8 + 1
        assert full["bytes_no_recompute"] - zero["bytes_no_recompute"] == pytest.approx(
            7 / 8 * full["head_optimizer_bytes"])
        # ZeRO-1 over DP = 2 (BASELINE config 5): the stage parameters' f32 master + Adam
        # moments (12 of their 20 bytes) halve per replica
        l4 = balanced_layer_ranges(cfg, 4, 8192, head_on_last=False)
        o4 = generate("1F1B", 4, 8, 1, "loop")[1]
        rep = plan_recompute(cfg, l4, [1], o4, 1, 8192, torch.device("cuda", 0))
        dpz = plan_recompute(cfg, l4, [1], o4, 1, 8192, torch.device("cuda", 0), stage_shards=2)
        nparams = cfg.layer_params() * (l4[1][1] - l4[1][0])
        assert rep["bytes_no_recompute"] - dpz["bytes_no_recompute"] == pytest.approx(6.0 * nparams)
        # f32 arenas: the f32 weights are the master and stay whole, only the Adam
        # moments (8 bytes) shard: 12 + 8/dp per parameter, so DP=2 saves 4 bytes, not 6
        rep32 = plan_recompute(cfg, l4, [1], o4, 1, 8192, torch.device("cuda", 0), dtype=torch.float32)
        dpz32 = plan_recompute(cfg, l4, [1], o4, 1, 8192, torch.device("cuda", 0), stage_shards=2,
                               dtype=torch.float32)
        assert rep32["bytes_no_recompute"] - dpz32["bytes_no_recompute"] == pytest.approx(4.0 * nparams)
        # HIP graphs: the captures of a stash slot share one pool (parallel/stash.py), so a
        # rank holds its schedule's in-flight stashes (rank 1 of 1F1B PP = 4: 3 = P - s) per
        # microbatch lane; MIPIPE_STASH_RING=0 (one private pool per graph): all 8
        g = plan_recompute(cfg, l4, [1], o4, 1, 8192, torch.device("cuda", 0), graphs=True)
        g2 = plan_recompute(cfg, l4, [1], o4, 1, 8192, torch.device("cuda", 0), graphs=True, lanes=2)
        assert rep["inflight"] == 3 and g["inflight"] == 3 and 3 <= g2["inflight"] <= 4
        import os
        os.environ["MIPIPE_STASH_RING"] = "0"
        try:
            g0 = plan_recompute(cfg, l4, [1], o4, 1, 8192, torch.device("cuda", 0), graphs=True)
        finally:
            del os.environ["MIPIPE_STASH_RING"]
        assert g0["inflight"] == 8 and g0["bytes_no_recompute"] > g2["bytes_no_recompute"]
        assert dpz32["bytes_no_recompute"] > dpz["bytes_no_recompute"]
        h32 = plan_recompute(cfg, l8, [7], o8, 1, 8192, torch.device("cuda", 0), head_tokens=1024, head_shards=8,
                             dtype=torch.float32)
        emb = cfg.vocab_padded * cfg.d_model
        assert h32["head_optimizer_bytes"] == pytest.approx(8.0 * emb / 8)
        assert h32["head_state_bytes"] == pytest.approx(12.0 * emb + 8.0 * emb / 8)
    finally:
        E.torch.cuda.get_device_properties = orig
    # 1F1B PP=4: rank 0 holds 4 microbatches in flight, the last rank 1; GPipe holds all m
    o4 = generate("1F1B", 4, 8, 1, "loop")
    assert max_inflight_microbatches(o4[0], {0}) == 4 and max_inflight_microbatches(o4[3], {3}) == 1
    assert max_inflight_microbatches(generate("GPipe", 4, 8, 1, "loop")[0], {0}) == 8


def _arena_worker(rank, world, split_head):
    cfg = CFG["gpt2"]()
    tr = PipelineTrainer(cfg, pp=world, schedule="1F1B", n_microbatches=M, mbs=MBS, seq_len=S,
                         device=torch.device("cpu"), dtype=torch.float32, layer_ranges=[(0, 2), (2, 4)],
                         split_head=split_head, head_align=8)
    rt = tr.runtime
    x, y = _data(cfg)
    tr.train_step(x, y)
    keys0 = set(rt._recv_bufs)
    ptrs0 = {k: [t.data_ptr() for t in v] for k, v in rt._recv_bufs.items()}
    lo = rt._recv_arena.data_ptr() if rt.recv_arena_bytes else 0
    hi = lo + rt.recv_arena_bytes
    inside = all(lo <= p < hi for ps in ptrs0.values() for p in ps)
    dh_inside = all(lo <= t.data_ptr() < hi for t in rt._dh_full.values())
    tr.train_step(x, y)
    same = set(rt._recv_bufs) == keys0 and ptrs0 == {k: [t.data_ptr() for t in v] for k, v in rt._recv_bufs.items()}
    return dict(bytes=rt.recv_arena_bytes, n=len(keys0), inside=inside, dh_inside=dh_inside, same=same,
                n_dh=len(rt._dh_full))


@pytest.mark.parametrize("split_head", [False, True])
def test_recv_arena_planned_up_front(split_head):
    """Every receive slot of the lowered program comes from the one arena planned at init
    (no lazy allocation inside the step, fixed addresses across steps)."""
    res = run_world(_arena_worker, 2, split_head)
    for r, o in res.items():
        assert o["bytes"] > 0 and o["n"] > 0, o
        assert o["inside"] and o["dh_inside"] and o["same"], o
    # stage 1 receives M activations; stage 0 receives M gradients (+ head chunks)
    assert res[0]["n"] >= M and res[1]["n"] >= M
    if split_head:
        assert res[1]["n_dh"] == M


def _zero_worker(rank, world, name, pp, dp, zero, split_head=True, save=None, load=None, reduce_dtype="f32"):
    import os
    os.environ["MIPIPE_DP_ZERO"] = "1" if zero else "0"
    os.environ["MIPIPE_DP_REDUCE_DTYPE"] = reduce_dtype
    cfg = CFG[name]()
    tr = PipelineTrainer(cfg, pp=pp, dp=dp, schedule="1F1B", n_microbatches=M, mbs=MBS, seq_len=S,
                         device=torch.device("cpu"), dtype=torch.float32, lr=1.0, adam_eps=1.0,
                         layer_ranges=[(0, 2), (2, 4)] if pp == 2 else None, split_head=split_head, head_align=8,
                         max_grad_norm=0.05)
    sharded = [st.arena.shard_scope for st in tr.stages]
    first = 0
    if load is not None:
        tr.load_checkpoint(load)
        first = 2
    losses = []
    for step in range(first, first + 2):
        x, y = _data(cfg, tr.mesh.dp_rank, step)
        l = tr.train_step(x, y)
        if l is not None:
            losses.append(float(l))
    if save is not None:
        tr.save_checkpoint(save)
    sd = {k: v.numpy().copy() for k, v in tr.state_dict().items()}
    m = [t.clone() for t in tr.optimizer.m]
    return dict(losses=losses, sd=sd, sharded=sharded, m_numel=[t.numel() for t in m],
                arena_numel=[st.arena.numel for st in tr.stages], dp_zero=tr.dp_zero)


@pytest.mark.parametrize("name,pp", [("llama", 2), ("gpt2", 1)])
def test_dp_zero1_matches_replicated_dp(name, pp):
    """ZeRO-1 over DP replicas (each replica keeps 1/dp of every stage arena's master and
    Adam moments; REDUCE_GRAD is a reduce-scatter, the step all-gathers the weights) gives
    the same weights and losses as the replicated optimizer, with the clip active."""
    world = 2 * pp
    on = run_world(_zero_worker, world, name, pp, 2, True)
    off = run_world(_zero_worker, world, name, pp, 2, False)
    for r in range(world):
        assert on[r]["dp_zero"] and not off[r]["dp_zero"]
        assert on[r]["sharded"] == ["dp"] * len(on[r]["sharded"])
        # this replica's moments cover 1/dp of its stage arenas
        for mn, an in zip(on[r]["m_numel"], on[r]["arena_numel"]):
            assert mn * 2 == an
        assert on[r]["losses"] == pytest.approx(off[r]["losses"], rel=1e-5)
        for k, v in on[r]["sd"].items():
            torch.testing.assert_close(torch.from_numpy(v), torch.from_numpy(off[r]["sd"][k]), atol=1e-5, rtol=1e-5,
                                       msg=lambda m: f"{k}: {m}")


def test_dp_bf16_reduce_scatter_tracks_f32():
    """MIPIPE_DP_REDUCE_DTYPE=bf16 (half the bytes of the DP gradient reduce-scatter): the
    replicas' weights stay identical and training tracks the f32 reduction to bf16
    rounding of the gradient."""
    world = 4
    f32 = run_world(_zero_worker, world, "gpt2", 2, 2, True, True, None, None, "f32")
    b16 = run_world(_zero_worker, world, "gpt2", 2, 2, True, True, None, None, "bf16")
    for r in range(world):
        assert b16[r]["losses"] == pytest.approx(f32[r]["losses"], rel=2e-2)
        for k, v in b16[r]["sd"].items():
            torch.testing.assert_close(torch.from_numpy(v), torch.from_numpy(f32[r]["sd"][k]), atol=3e-2, rtol=3e-2)
    for r in range(2):   # DP peers (ranks r and r + pp) hold the same stage weights
        for k, v in b16[r]["sd"].items():
            assert (v == b16[r + 2]["sd"][k]).all(), k
    # ... and the bf16 path did run: the rounding shows up somewhere
    assert any((v != f32[r]["sd"][k]).any() for r in range(world) for k, v in b16[r]["sd"].items())


def test_dp_zero1_checkpoint_resume(tmp_path):
    """A DP=2 x PP=2 ZeRO-1 run saved after 2 steps and resumed (collective gather of the
    sharded masters / moments) continues exactly like the uninterrupted 4-step run."""
    path = str(tmp_path / "ck")
    full = run_world(_zero_worker, 4, "llama", 2, 2, True)
    # the uninterrupted oracle: 4 steps in one run
    ref = run_world(_four_steps_worker, 4)
    run_world(_zero_worker, 4, "llama", 2, 2, True, True, path)
    res = run_world(_zero_worker, 4, "llama", 2, 2, True, True, None, path)
    assert full[0]["dp_zero"]
    for r in range(4):
        for k, v in res[r]["sd"].items():
            torch.testing.assert_close(torch.from_numpy(v), torch.from_numpy(ref[r][k]), atol=1e-5, rtol=1e-5,
                                       msg=lambda m: f"{k}: {m}")


def _four_steps_worker(rank, world):
    import os
    os.environ["MIPIPE_DP_ZERO"] = "1"
    cfg = CFG["llama"]()
    tr = PipelineTrainer(cfg, pp=2, dp=2, schedule="1F1B", n_microbatches=M, mbs=MBS, seq_len=S,
                         device=torch.device("cpu"), dtype=torch.float32, lr=1.0, adam_eps=1.0,
                         layer_ranges=[(0, 2), (2, 4)], split_head=True, head_align=8, max_grad_norm=0.05)
    for step in range(4):
        x, y = _data(cfg, tr.mesh.dp_rank, step)
        tr.train_step(x, y)
    return {k: v.numpy().copy() for k, v in tr.state_dict().items()}


def test_trainer_auto_schedule():
    """PipelineTrainer(schedule="auto") (train.py's `parallel.schedule: auto`): the best
    head-aware plan -- 1F1B on one stage; at PP > 1 the same choice as pick_schedule."""
    from mipipe.engine import PipelineTrainer, pick_schedule
    from mipipe.models.config import NativeConfig
    cfg = NativeConfig.by_name("gpt2-tiny", vocab_size=256)
    tr = PipelineTrainer(cfg, pp=1, schedule="auto", n_microbatches=2, mbs=2, seq_len=16, device="cpu")
    assert tr.schedule == "1F1B" and tr.schedule_choice == {}
    name, eff = pick_schedule(NativeConfig.by_name("gpt2-small"), 2, 8, 32, 1024)
    beats = [k for k in eff if k != "1F1B" and eff[k] >= eff["1F1B"] * 1.01]
    assert name in eff and (name == max(beats, key=lambda k: eff[k]) if beats else name == "1F1B"), (name, eff)


def test_pick_microbatch_uses_rates_measured_for_the_model():
    """--mbs auto scores each candidate with the kernel rate measured for the
    model's own per-rank shapes (bench.py --phase rate on engine.rate_probe_config) when
    given, the GPT-2-small table otherwise."""
    from mipipe.engine import pick_microbatch, rate_probe_config
    from mipipe.models.config import NativeConfig
    cfg = NativeConfig.gpt2("small")
    mbs, m, sc = pick_microbatch(cfg, 4, 1024, 512, rates={32: 1.0e6, 16: 1.0e6})
    assert sc[16]["rate_source"] == "measured" and sc[16]["kernel_rate"] == 1.0
    assert mbs == 16 and m == 32      # same per-token rate: the smaller bubble wins
    mbs, m, sc = pick_microbatch(cfg, 4, 1024, 512, rates={"32": 1.0e6, "16": 0.5e6})
    assert mbs == 32 and sc[16]["kernel_rate"] == 0.5 and sc[32]["rate_source"] == "measured"
    p = rate_probe_config(NativeConfig.llama3("8b"), 8)
    assert p.n_layers == 4 and p.vocab_size >= 128256 // 8 and p.vocab_size % 128 == 0
    assert p.vocab_padded >= p.vocab_size


def test_first_step_comm_audit_passes_on_every_rank():
    """the first step's issued p2p (per pair and channel, in order) and
    collectives (per group) agree across all ranks -- DP = 2 x PP = 2 with the distributed
    head exercises pipeline p2p, the head reductions, the DP gradient and the clip norm."""
    res = run_world(_worker, 4, "gpt2", 2, 2, "1F1B", True)
    for r in range(4):
        a = res[r]["audit"]
        assert a is not None and a["ok"] and a["problems"] == [], (r, a)
        assert a["entries"] > 0


def test_comm_audit_finds_order_and_collective_mismatches():
    """parallel/audit.check: a send order that differs from the receiver's, a missing
    receive and a collective sequence that differs within its group are each reported."""
    from mipipe.parallel.audit import check
    f32 = "float32"
    ok = {0: [("p2p", 0, ((1, 64, f32),), ()), ("p2p", 0, ((1, 32, f32),), ()),
              ("coll", "pp", (0, 1), "all_reduce_sum", 8, f32)],
          1: [("p2p", 0, (), ((0, 64, f32),)), ("p2p", 0, (), ((0, 32, f32),)),
              ("coll", "pp", (0, 1), "all_reduce_sum", 8, f32)]}
    assert check(ok) == []
    swapped = {0: ok[0], 1: [ok[1][1], ok[1][0], ok[1][2]]}
    p = check(swapped)
    assert len(p) == 1 and p[0].startswith("p2p 0->1 channel 0") and "#0" in p[0], p
    missing = {0: ok[0], 1: [ok[1][0], ok[1][2]]}
    assert any("2 sends vs 1 receives" in x for x in check(missing))
    coll = {0: ok[0], 1: ok[1][:2] + [("coll", "pp", (0, 1), "all_gather", 8, f32)]}
    assert any(x.startswith("pp collectives over [0, 1]") for x in check(coll))
    # another channel is another match queue
    ch = {0: [("p2p", 1, ((1, 64, f32),), ())], 1: [("p2p", 0, (), ((0, 64, f32),))]}
    assert len(check(ch)) == 2


def test_schedule_margin_depends_on_traffic():
    """pick_schedule: a candidate that sends exactly 1F1B's messages (ZBH1, GPipe, v = 1
    interleaved) needs a 1 % better plan, one that sends more (interleaved v > 1) 3 %.
    GPT-2 small at P = 8 with 16-sequence microbatches: ZBH1 plans 2.7 % over 1F1B and is
    taken; with a 3 % margin for every candidate it would not be."""
    from mipipe.engine import pick_schedule
    from mipipe.models.config import NativeConfig
    cfg = NativeConfig.by_name("gpt2-small")
    name, eff = pick_schedule(cfg, 8, 64, 16, 1024, candidates=("1F1B", "ZBH1"))
    assert 1.01 <= eff["ZBH1"] / eff["1F1B"] < 1.03 and name == "ZBH1", eff
    name3, _ = pick_schedule(cfg, 8, 64, 16, 1024, candidates=("1F1B", "ZBH1"), same_traffic_margin=0.03)
    assert name3 == "1F1B"
    # interleaved with two chunks per rank sends twice the activations: the full margin
    name_i, eff_i = pick_schedule(cfg, 2, 8, 32, 1024, candidates=("1F1B", "Interleaved1F1B"))
    assert eff_i["Interleaved1F1B"] < eff_i["1F1B"] * 1.03 and name_i == "1F1B", eff_i



def test_selective_recompute_picks_the_fewest_layers_that_fit():
    """recompute="auto" recomputes the fewest layers per stage whose plan fits
    the budget: 0 when the stash fits, every layer only when nothing less does, and the
    bytes fall monotonically with k.  Llama-3 8B, seq 8192, one MI355X: GPipe m = 4 (4
    stashes of 32 layers) needs some layers recomputed, 1F1B m = 2 none."""
    import torch
    from mipipe.engine import plan_recompute
    from mipipe.models.config import NativeConfig
    from mipipe.models.native import balanced_layer_ranges
    from mipipe.parallel.schedules import generate
    cfg = NativeConfig.llama3("8b")
    lr = balanced_layer_ranges(cfg, 1, 8192, head_on_last=True)
    hbm = 288 * 2 ** 30
    p1 = plan_recompute(cfg, lr, [0], generate("1F1B", 1, 2, 1)[0], 1, 8192, torch.device("cpu"),
                        head_tokens=8192, hbm=hbm)
    assert p1["recompute_layers"] == 0 and not p1["recompute"]
    p4 = plan_recompute(cfg, lr, [0], generate("GPipe", 1, 4, 1)[0], 1, 8192, torch.device("cpu"),
                        head_tokens=8192, hbm=hbm)
    k = p4["recompute_layers"]
    assert p4["recompute"] and 0 < k < 32, k
    f = p4["selective_fn"]
    assert f(k) <= 0.85 * hbm < f(k - 1)
    assert all(f(i + 1) < f(i) for i in range(32))
    assert f(32) == pytest.approx(p4["bytes_recompute"]) and f(0) == p4["bytes_no_recompute"]
    # nothing fits: every layer
    p_small = plan_recompute(cfg, lr, [0], generate("GPipe", 1, 4, 1)[0], 1, 8192, torch.device("cpu"),
                             head_tokens=8192, hbm=64 * 2 ** 30)
    assert p_small["recompute_layers"] == 32


def test_pick_schedule_records_lags_and_bounds_the_stash_by_hbm():
    """every candidate of schedule="auto" is planned under the HBM bound and
    its record carries the head lag it assumed, its largest per-rank stash and planned GB.
    GPT-2 small at P = 8 (16K-token microbatches): whatever wins fits with margin.  Llama-3
    8B at P = 8 on a hypothetical 64 GB device: no candidate keeps a lag whose stash would
    not fit -- the lag falls back toward the schedule's own depth (ZBH1: <= P + lanes slots)."""
    from mipipe.engine import pick_schedule
    from mipipe.models.config import NativeConfig
    det = {}
    name, eff = pick_schedule(NativeConfig.gpt2("small"), 8, 64, 16, 1024, details=det)
    assert set(det) == set(eff) and name in det
    for c, d in det.items():
        assert {"head_lag", "stash_slots_max", "planned_gb_max", "efficiency", "v"} <= set(d), d
        assert d["planned_gb_max"] <= 0.85 * 288 * 2 ** 30 / 1e9, (c, d)
    cfg = NativeConfig.llama3("8b")
    bound = {"hbm": 64 * 2 ** 30, "lanes": 2}
    det8 = {}
    pick_schedule(cfg, 8, 16, 1, 8192, candidates=("1F1B", "ZBH1"), mem_bound=bound, details=det8)
    free = {}
    pick_schedule(cfg, 8, 16, 1, 8192, candidates=("1F1B", "ZBH1"), details=free)
    for c in ("1F1B", "ZBH1"):
        d, f = det8[c], free[c]
        assert d["head_lag"] <= f["head_lag"], (c, d, f)
        fits = d["planned_gb_max"] <= 0.85 * 64 * 2 ** 30 / 1e9
        # either the plan fits the small device, or it could not shrink below the schedule's
        # own warmup depth (lag 0)
        assert fits or d["head_lag"] == 0, (c, d)
    assert det8["ZBH1"]["head_lag"] == 0 or det8["ZBH1"]["stash_slots_max"] <= 8 + 2, det8
