"""Pure-Python schedule tests (SURVEY §4 tier 1): golden IR, validator, lowering
deadlock-freedom under RCCL semantics, analytic vs simulated bubble."""
import itertools

import pytest

import mipipe  # noqa: F401
from mipipe.parallel import Action, Op, analytic_bubble, generate, lower, simulate
from mipipe.parallel.ir import CommGroup, from_csv, to_csv
from mipipe.parallel.schedules import stage_to_rank
from mipipe.parallel.simulate import check_lowered
from mipipe.parallel.validate import ScheduleError, validate


def seq(s):
    return [Action.parse(x) for x in s.split()]


def test_action_roundtrip():
    for s in ["2F0", "1SEND_B3", "0REDUCE_GRAD", "12W7", "3RECV_F10"]:
        assert str(Action.parse(s)) == s
    with pytest.raises(ValueError):
        Action.parse("xF0")


def test_gpipe_golden():
    # rank r runs rF0..rF3 rB0..rB3
    o = generate("GPipe", 2, 4)
    assert o[1] == seq("1F0 1F1 1F2 1F3 1B0 1B1 1B2 1B3")


def test_1f1b_execution_order():
    # dependency schedules.py:873-994 execution order for PP=4, m=4
    o = generate("1F1B", 4, 4)
    assert o[0] == seq("0F0 0F1 0F2 0F3 0B0 0B1 0B2 0B3")
    assert o[3] == seq("3F0 3B0 3F1 3B1 3F2 3B2 3F3 3B3")
    assert o[1] == seq("1F0 1F1 1F2 1B0 1F3 1B1 1B2 1B3")


def test_interleaved_golden_appendix_a():
    o = generate("Interleaved1F1B", 2, 4, 2)
    assert o[0] == seq("0F0 0F1 2F0 2F1 0F2 2B0 0F3 2B1 2F2 0B0 2F3 0B1 2B2 2B3 0B2 0B3")
    assert o[1] == seq("1F0 1F1 3F0 3B0 3F1 3B1 1F2 1B0 1F3 1B1 3F2 3B2 3F3 3B3 1B2 1B3")


def test_interleaved_m_equals_p_is_fill_drain_like():
    # PP=4, v=2, m=4 -> every rank does all 8 forwards first
    o = generate("Interleaved1F1B", 4, 4, 2)
    assert all(a.op == Op.F for a in o[0][:8])


CASES = [(n, P, m, v) for n, v in [("GPipe", 1), ("1F1B", 1), ("Interleaved1F1B", 2), ("Interleaved1F1B", 3),
                                    ("LoopedBFS", 2), ("ZBH1", 1)]
         for P in (1, 2, 4, 8) for m in (P, 2 * P, 4 * P, 4)]


@pytest.mark.parametrize("name,P,m,v", CASES)
def test_validate_lower_and_no_deadlock(name, P, m, v):
    if name == "Interleaved1F1B" and m % max(1, m // P):
        pytest.skip("torch-style interleave requires m % rounds == 0")
    o = generate(name, P, m, v)
    validate(o, P, v, m)
    prog = lower(o, P, v)  # runs check_lowered (one comm stream per rank)
    # the native engine's per-direction channels (2 comm streams per rank) must be safe too,
    # also with receive-only posts started at post time
    check_lowered(prog, P * v, channels=2)
    check_lowered(prog, P * v, channels=2, recv_early=True)
    # every send has exactly one matching recv with the same key, posted by the peer
    sends, recvs = {}, {}
    for r, es in prog.items():
        for e in es:
            if not isinstance(e, Action):
                for op in e.ops:
                    (sends if op.action.op.is_send else recvs)[op.key] = (r, op.peer)
    assert set(sends) == set(recvs)
    for k, (r, peer) in sends.items():
        assert recvs[k] == (peer, r)
    # one REDUCE_GRAD per stage
    rg = [e for es in prog.values() for e in es if isinstance(e, Action) and e.op == Op.REDUCE_GRAD]
    assert sorted(a.stage for a in rg) == list(range(P * v))


def test_validator_catches_errors():
    o = generate("1F1B", 2, 4)
    bad = {0: o[0][:-1], 1: o[1]}
    with pytest.raises(ScheduleError):
        validate(bad, 2, 1, 4)
    swapped = {0: o[0], 1: [o[1][1], o[1][0]] + o[1][2:]}
    with pytest.raises(ScheduleError):
        validate(swapped, 2, 1, 4)


def test_checker_detects_deadlock():
    # hand-built program where both ranks send before receiving in separate groups in
    # crossed order -> must be rejected
    from mipipe.parallel.ir import CommGroup, CommOp
    prog = {
        0: [Action(0, Op.F, 0), CommGroup([CommOp(Action(0, Op.RECV_B, 0), 1, ("B", 0, 0))]),
            CommGroup([CommOp(Action(0, Op.SEND_F, 0), 1, ("F", 1, 0))]), Action(0, Op.B, 0)],
        1: [CommGroup([CommOp(Action(1, Op.RECV_F, 0), 0, ("F", 1, 0))]), Action(1, Op.F, 0), Action(1, Op.B, 0),
            CommGroup([CommOp(Action(1, Op.SEND_B, 0), 0, ("B", 0, 0))])],
    }
    with pytest.raises(RuntimeError):
        check_lowered(prog, 2)
    # with one comm stream per direction the early gradient receive no longer holds back
    # the activation send: the same program is safe on the native engine's 2 channels
    check_lowered(prog, 2, channels=2)


def test_pp8_interleaved_v2_m16_gpt2_medium_lowering():
    """BASELINE config 3 (configs/gpt2_medium_interleaved_pp8.yaml): GPT-2 medium,
    Interleaved 1F1B, PP=8, v=2, m=16, distributed head -- the exact program the runtime
    builds must validate, lower and be hang-free on 1 and 2 comm channels, with the
    simulated bubble of the plain schedule equal to the analytic (P-1)/(v*m+P-1)."""
    from mipipe.models.config import NativeConfig
    from mipipe.models.native import balanced_layer_ranges, stage_cost_model
    from mipipe.parallel.headsplit import head_token_split, plan_head_schedule
    P, v, m = 8, 2, 16
    base = generate("Interleaved1F1B", P, m, v)
    validate(base, P, v, m)
    assert simulate(base, P, v).bubble == pytest.approx((P - 1) / (v * m + P - 1), abs=1e-9)
    cfg = NativeConfig.gpt2("medium")
    lr = balanced_layer_ranges(cfg, P * v, 1024, head_on_last=False, ranks=P)
    assert len(lr) == 16 and lr[0][0] == 0 and lr[-1][1] == 24
    lc, head_units, ec = stage_cost_model(cfg, 1024)
    stage_costs = [(b - a) * lc + (ec if s == 0 else 0.0) for s, (a, b) in enumerate(lr)]
    rank_load = [sum(stage_costs[s] for s in range(P * v) if s % P == r) for r in range(P)]
    chunks = head_token_split(8 * 1024, rank_load, head_units, align=256)
    assert sum(chunks) == 8 * 1024
    head_costs = {r: 3.0 * head_units * chunks[r] / (8 * 1024) for r in range(P) if chunks[r] > 0}
    # rank-balanced split (every rank 3 layers; no empty virtual stage) and the planner's
    # deeper-warmup regeneration, as plan_head_pipeline runs it
    assert all(b > a for a, b in lr)
    orders, lag, makespan = plan_head_schedule(base, P, v, "loop", head_costs, stage_costs,
                                               regen=lambda k: generate("Interleaved1F1B", P, m, v, warmup_extra=k))
    validate(orders, P, v, m)
    prog = lower(orders, P, v, "loop", head_costs=head_costs, stage_costs=stage_costs)
    check_lowered(prog, P * v, channels=1)
    check_lowered(prog, P * v, channels=2)
    ideal = (3.0 * sum(stage_costs) + sum(head_costs.values())) * m / P
    assert ideal / makespan > 0.70, (ideal, makespan, lag)


@pytest.mark.parametrize("P,m", [(2, 4), (4, 4), (4, 8), (8, 16)])
def test_bubble_analytic_matches_simulation(P, m):
    for name in ("GPipe", "1F1B"):
        sim = simulate(generate(name, P, m), P)
        assert sim.bubble == pytest.approx(analytic_bubble(name, P, m), abs=1e-9)
    sim = simulate(generate("Interleaved1F1B", P, 2 * P, 2), P, 2)
    assert sim.bubble == pytest.approx(analytic_bubble("Interleaved1F1B", P, 2 * P, 2), abs=1e-9)


def test_zero_bubble_beats_1f1b():
    for P, m in [(4, 8), (8, 16)]:
        assert simulate(generate("ZBH1", P, m), P).bubble < simulate(generate("1F1B", P, m), P).bubble


def test_csv_roundtrip_and_placement():
    o = generate("Interleaved1F1B", 4, 8, 2)
    assert from_csv(to_csv(o)) == o
    assert [stage_to_rank(s, 4, "v") for s in range(8)] == [0, 1, 2, 3, 3, 2, 1, 0]
    assert [stage_to_rank(s, 4, "loop") for s in range(8)] == [0, 1, 2, 3, 0, 1, 2, 3]


def test_v_placement_interleaved_lowering():
    with pytest.raises(ValueError):
        generate("Interleaved1F1B", 4, 8, 2, style="v")
    o = generate("LoopedBFS", 4, 8, 2, style="v")
    validate(o, 4, 2, 8, style="v")
    prog = lower(o, 4, 2, style="v")
    # the chunk boundary 3 -> 4 is on the same rank under 'v': no comm for it
    keys = {op.key for es in prog.values() for e in es if not isinstance(e, Action) for op in e.ops}
    assert ("F", 4, 0) not in keys


# ----------------------------------------------------------------------------- distributed head
from mipipe.parallel.headsplit import head_token_split, insert_head_ops, plan_head_schedule  # noqa: E402


def test_head_token_split_levels_load():
    load = [1.1, 1, 1, 1, 2, 2, 2, 2.1]
    tok = head_token_split(16384, load, 5.2, align=128)
    assert sum(tok) == 16384 and all(t % 128 == 0 for t in tok)
    tot = [l + 5.2 * t / 16384 for l, t in zip(load, tok)]
    assert max(tot) - min(tot) < 0.1
    # a rank already above the water level gets nothing
    assert head_token_split(1024, [0, 0, 10], 1.0, align=128)[2] == 0


@pytest.mark.parametrize("P", [2, 3, 4, 8])
@pytest.mark.parametrize("sched", ["1F1B", "GPipe", "ZBH1", "Interleaved1F1B", "LoopedBFS"])
def test_head_ops_lower_without_deadlock(P, sched):
    from mipipe.parallel.schedules import SCHEDULES
    v = 2 if SCHEDULES[sched][2] else 1
    m = 2 * P
    for skew in (0.0, 1.0):
        hc = {r: 0.5 + skew * r / P for r in range(P)}
        if skew:
            hc.pop(1 % P, None)   # a rank without a chunk
        orders = generate(sched, P, m, v, "loop")
        ho, lag, mk = plan_head_schedule(orders, P, v, "loop", hc)
        validate(ho, P, v, m, "loop")
        for r in range(P):
            hs = [a.mb for a in ho[r] if a.op == Op.H]
            assert hs == (list(range(m)) if r in hc else [])
        prog = lower(ho, P, v, "loop", head_costs=hc)   # runs the RCCL-semantics deadlock check
        kinds = {op.key[0] for es in prog.values() for e in es if isinstance(e, CommGroup) for op in e.ops}
        assert {"H", "D"} <= kinds


def test_head_split_beats_last_stage_head_in_simulation():
    """GPT-2 small PP=8: the distributed head removes the last-stage bottleneck."""
    P, m, head = 8, 16, 5.2
    load = [1.1, 1, 1, 1, 2, 2, 2, 2.1]
    tok = head_token_split(16384, load, head)
    hc = {r: 3 * head * t / 16384 for r, t in enumerate(tok) if t}
    o = generate("1F1B", P, m, 1, "loop")
    base = simulate(o, P, 1, "loop", stage_costs=[c + (head if s == P - 1 else 0) for s, c in enumerate(load)])
    _, _, mk = plan_head_schedule(o, P, 1, "loop", hc, stage_costs=load)
    assert mk < 0.6 * base.makespan


@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_zbv_valid_lowerable_and_low_bubble(P):
    m = 2 * P
    o = generate("ZBV", P, m, 2, "v")
    validate(o, P, 2, m, "v")
    lower(o, P, 2, "v")
    for r in range(P):   # V placement: rank r holds stages r and 2P-1-r
        assert {a.stage for a in o[r]} == {r, 2 * P - 1 - r}
    zbv = simulate(o, P, 2, "v", stage_costs=[0.5] * (2 * P)).bubble
    f1b = simulate(generate("1F1B", P, m, 1, "loop"), P, 1, "loop").bubble
    assert zbv < 0.6 * f1b


# ----------------------------------------------------------------------------- deeper warmup
@pytest.mark.parametrize("name,v", [("1F1B", 1), ("Interleaved1F1B", 2)])
@pytest.mark.parametrize("P,m", [(2, 4), (4, 4), (4, 16), (8, 32)])
def test_warmup_extra_orders_valid_and_hang_free(name, v, P, m):
    """Every extra-warmup depth (0 = torch's order, large = all forwards first) gives a
    valid, lowerable order with the same ideal-uniform bubble or better."""
    base = simulate(generate(name, P, m, v), P, v).makespan
    for extra in (0, 1, 2, 5, m * v):
        o = generate(name, P, m, v, warmup_extra=extra)
        validate(o, P, v, m)
        check_lowered(lower(o, P, v), P * v)
        assert simulate(o, P, v).makespan <= base + 1e-9
    assert generate(name, P, m, v, warmup_extra=0) == generate(name, P, m, v)


def test_interleaved_m_equals_p_bubble_is_the_interleaved_ideal():
    """at m == P == 4, v = 2 torch's order runs every forward
    before the first backward on rank 0 -- but the simulated bubble is the interleaved
    ideal (P-1)/(v*m+P-1) = 0.273, not GPipe's 0.429: the fill-drain shape costs stash
    (m*v chunk activations per rank, i.e. m stage-equivalents, as GPipe), not time."""
    P, m, v = 4, 4, 2
    o = generate("Interleaved1F1B", P, m, v)
    assert [a.op for a in o[0][:m * v]] == [Op.F] * (m * v)
    sim = simulate(o, P, v)
    assert sim.bubble == pytest.approx(3 / 11, abs=1e-9) and sim.bubble <= 0.30
    assert simulate(generate("GPipe", P, m), P).bubble == pytest.approx(3 / 7, abs=1e-9)


@pytest.mark.parametrize("P", [2, 4, 8])
def test_interleaved_with_head_plans_ahead_of_1f1b_and_gpipe(P):
    """GPT-2 small, m = 4P (bench.py's pipeline config), distributed head: the planner's
    regenerated deeper-warmup interleaved order beats 1F1B and GPipe in planned efficiency
    (without regeneration the lag re-sort deadlocks interleaved orders and only lag 0 was
    feasible: 0.845 at P=2, below 1F1B's 0.912)."""
    from mipipe.models.config import NativeConfig
    from mipipe.models.native import balanced_layer_ranges, stage_cost_model
    from mipipe.parallel.schedules import WARMUP_EXTRA
    cfg = NativeConfig.gpt2("small")
    m, seq, T = 4 * P, 1024, 32 * 1024
    eff = {}
    for name, v in (("GPipe", 1), ("1F1B", 1), ("Interleaved1F1B", 2)):
        S = P * v
        lr = balanced_layer_ranges(cfg, S, seq, head_on_last=False, ranks=P)
        lc, hu, ec = stage_cost_model(cfg, seq)
        sc = [(b - a) * lc + (ec if s == 0 else 0.0) + (0.1 if s == S - 1 else 0.0) for s, (a, b) in enumerate(lr)]
        load = [sum(sc[s] for s in range(S) if s % P == r) for r in range(P)]
        ch = head_token_split(T, load, hu, align=256)
        hc = {r: 3.0 * hu * ch[r] / T for r in range(P) if ch[r] > 0}
        regen = (lambda lag, name=name, v=v: generate(name, P, m, v, warmup_extra=lag)) if name in WARMUP_EXTRA \
            else None
        o, lag, mk = plan_head_schedule(generate(name, P, m, v), P, v, "loop", hc, sc, regen=regen)
        validate(o, P, v, m)
        check_lowered(lower(o, P, v, "loop", head_costs=hc, stage_costs=sc), S)
        eff[name] = (3.0 * sum(sc) + sum(hc.values())) * m / P / mk
    assert eff["Interleaved1F1B"] > max(eff["1F1B"], eff["GPipe"]) + 0.02, eff
    # 1F1B may give up to the head planner's lag tolerance (1 %) for a smaller stash
    assert eff["1F1B"] >= eff["GPipe"] * (1 - 0.01) - 1e-6, eff


@pytest.mark.parametrize("name,v", [("GPipe", 1), ("1F1B", 1), ("Interleaved1F1B", 2)])
@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("dp", [1, 2])
def test_overlapped_programs_proven_with_and_without_lanes(name, v, P, dp):
    """every PP x DP x schedule program with its collectives left in place
    (REDUCE_GRAD right after the stage's last backward, REDUCE_HEAD after the last head
    chunk) passes the independent-queue model on 1 and 2 channels, and with two
    microbatch lanes per rank; the deferred placement passes the serial model."""
    from mipipe.parallel.lower import add_head_reduce, defer_collectives
    m = 4 * P
    orders = generate(name, P, m, v)
    hc = {r: 0.5 for r in range(P)}
    ho, _, _ = plan_head_schedule(orders, P, v, "loop", hc)
    prog = add_head_reduce(lower(ho, P, v, "loop", head_costs=hc))
    for ch in (1, 2):
        for lanes in (1, 2):
            for early in (False, True):
                check_lowered(prog, P * v, channels=ch, dp=dp, lanes=lanes, recv_early=early)
    check_lowered(defer_collectives(prog), P * v, serial=True, dp=dp)


def test_recv_early_lets_a_receive_start_before_earlier_compute():
    """check_lowered(recv_early=True) models a receive-only post as starting at post time
    (its start no longer waits for the rank's earlier compute, only for its channel queue).
    1F1B's lowered program has such pre-posted receives; it is proven with them in the
    independent model, and the serial model (one FIFO per rank) is unaffected."""
    from mipipe.parallel.lower import lower as _lower
    from mipipe.parallel.ir import CommGroup
    P, m = 2, 4
    prog = _lower(generate("1F1B", P, m, 1), P, 1)
    recv_only = [e for es in prog.values() for e in es if isinstance(e, CommGroup)
                 and all(op.action.op.is_recv for op in e.ops)]
    assert recv_only, "1F1B's lowered program has receive-only groups (pre-posted receives)"
    check_lowered(prog, P, channels=2, recv_early=True)
    check_lowered(prog, P, serial=True, recv_early=True)   # no effect on the serial model


def test_microbatch_rate_interpolates_the_measured_table():
    from mipipe.engine import MICROBATCH_RATE, microbatch_rate
    assert microbatch_rate(32768) == 1.0 and microbatch_rate(1 << 20) == MICROBATCH_RATE[0][1]
    assert microbatch_rate(1024) == MICROBATCH_RATE[-1][1]
    r = [microbatch_rate(t) for t in (8192, 12000, 16384, 24000, 32768, 65536)]
    assert r == sorted(r), r          # more rows per kernel never plans slower


def test_pick_microbatch_weak_scaling_gpt2_small():
    """--mbs auto: smaller microbatches shrink the bubble but run each kernel on fewer rows;
    the larger candidate stays unless the smaller one scores > 2 % better (planned
    efficiency x measured kernel rate).  The batch per replica is fixed (128 P sequences).
    With the zero-bubble ZBH1 among the schedule candidates, GPT-2 small keeps
    32-sequence microbatches and runs ZBH1 at P = 2 / 4."""
    from mipipe.engine import pick_microbatch
    from mipipe.models.native import NativeConfig
    cfg = NativeConfig.by_name("gpt2-small")
    for P in (2, 4):
        mbs, m, sc = pick_microbatch(cfg, P, 1024, 128 * P)
        assert set(sc) == {32, 16} and mbs * m == 128 * P
        assert sc[16]["planned_efficiency"] > sc[32]["planned_efficiency"]      # the smaller bubble
        if mbs == 32:
            assert sc[16]["score"] <= 1.02 * sc[32]["score"]
        else:
            assert sc[16]["score"] > 1.02 * sc[32]["score"]
        assert sc[mbs]["schedule"] == "ZBH1", sc
    # without ZBH1's bubble filling, 16-sequence microbatches win at P = 4 (1F1B 0.92 vs 0.85)
    import mipipe.engine as E
    orig = E.pick_schedule
    try:
        E.pick_schedule = lambda *a, **k: orig(*a, candidates=("GPipe", "1F1B", "Interleaved1F1B"), **k)
        mbs, m, sc = pick_microbatch(cfg, 4, 1024, 512)
        assert (mbs, m) == (16, 32) and sc[16]["score"] > 1.02 * sc[32]["score"]
    finally:
        E.pick_schedule = orig


def test_stash_slot_plan_follows_the_schedule():
    """parallel/stash.py: the slots a stage's forwards occupy = the schedule's in-flight
    stashes -- 1F1B P - s (torch Schedule1F1B warmup, schedules.py:873-876), GPipe m, ZBH1
    until each W; never shared across microbatch lanes; a slot is reused only after its
    previous occupant's last reader."""
    from mipipe.parallel.ir import Op
    from mipipe.parallel.stash import plan_stash_slots, stash_slots_per_stage
    P, m = 4, 16
    for name, v in (("1F1B", 1), ("GPipe", 1), ("ZBH1", 1), ("Interleaved1F1B", 2)):
        orders = generate(name, P, m, v)
        for r in range(P):
            stages = [s for s in range(P * v) if s % P == r]
            for lanes in (1, 2):
                slot, last, count = plan_stash_slots(orders[r], stages, lanes)
                # replay: a slot is free again only after the last reader of its occupant
                held = {}
                for a in orders[r]:
                    if a is None or a.stage not in stages or a.mb is None:
                        continue
                    if a.op == Op.F:
                        k = (a.stage,) + slot[(a.stage, a.mb)]
                        assert k not in held, (name, r, a)
                        assert k[1] == a.mb % lanes
                        held[k] = a.mb
                    if last.get((a.stage, a.mb)) == a.op.value:
                        k = (a.stage,) + slot[(a.stage, a.mb)]
                        assert held.pop(k) == a.mb
                assert not held
            n = stash_slots_per_stage(orders[r], stages, 1)
            if name == "1F1B":
                assert n == {r: P - r}, (r, n)
            if name == "GPipe":
                assert n == {r: m}
            if name == "ZBH1":
                assert P - r <= n[r] < m


def test_head_plan_takes_the_smallest_lag_within_tolerance():
    """A head lag of m turns 1F1B's stash into GPipe's: the plan takes the smallest lag whose
    makespan is within lag_tol of the best, and honours max_lag."""
    from mipipe.engine import plan_head_pipeline
    from mipipe.models.config import NativeConfig
    from mipipe.parallel.headsplit import plan_head_schedule
    cfg = NativeConfig.gpt2("tiny", vocab_size=1000, d_model=256, n_layers=4, n_heads=4, d_ff=1024, max_seq_len=256)
    P, m = 4, 16
    base = plan_head_pipeline(cfg, P, "1F1B", m, 2, 256)
    sc, hc = base["stage_costs"], base["head_costs"]
    o = generate("1F1B", P, m, 1)
    _, lag_best, mk_best = plan_head_schedule(o, P, 1, "loop", hc, sc, comm=base["comm"], lag_tol=0.0)
    _, lag_loose, mk_loose = plan_head_schedule(o, P, 1, "loop", hc, sc, comm=base["comm"], lag_tol=10.0)
    assert lag_loose == 0 and lag_best > 0 and mk_loose >= mk_best
    _, lag_cap, mk_cap = plan_head_schedule(o, P, 1, "loop", hc, sc, comm=base["comm"], max_lag=2)
    assert lag_cap <= 2 and mk_cap >= mk_best
    # the cap shows in the stash plan: rank 0 holds fewer microbatches
    from mipipe.parallel.stash import stash_slots_per_stage
    full = plan_head_pipeline(cfg, P, "1F1B", m, 2, 256)["orders"]
    cap = plan_head_schedule(o, P, 1, "loop", hc, sc, comm=base["comm"], max_lag=0)[0]
    assert sum(stash_slots_per_stage(cap[0], [0], 1).values()) < sum(stash_slots_per_stage(full[0], [0], 1).values())
