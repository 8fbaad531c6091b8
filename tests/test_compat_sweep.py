"""Reference-compatible experiment API: the notebook's launcher,
sweep, speedup/efficiency analysis, pivot table, plots and environment report, on
CPU/gloo (the reference's own configuration), both engines."""
import os

import pytest

import mipipe  # noqa: F401
from mipipe.bench import compat


@pytest.mark.parametrize("engine", ["torch", "native"])
def test_run_one_experiment(engine, monkeypatch):
    # spawned ranks re-import torch; under a parallel test run (xdist) with every rank
    # taking all cores this took > 300 s: two threads per rank and a longer deadline
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    m = compat.run_one_experiment(4, 4, 2, "1F1B", batch_size=8, seq_length=16, num_iterations=1, device="cpu",
                                  engine=engine, timeout=900)
    assert "error" not in m, m
    assert m["tokens_processed"] == 8 * 16 * 1 and m["throughput"] > 0


def test_unknown_schedule_reports_error():
    m = compat.run_one_experiment(4, 4, 2, "NoSuchSchedule", batch_size=8, seq_length=16, num_iterations=1,
                                  device="cpu", timeout=120)
    assert "error" in m


def test_sweep_analysis_tables_and_plots(tmp_path):
    df = compat.run_all_experiments(n_heads_list=(4,), n_layers_list=(4,), num_processes_list=(2,),
                                    schedules=("GPipe", "1F1B", "Interleaved1F1B"), num_iterations=1,
                                    batch_size=8, seq_length=16, device="cpu", timeout=300)
    assert len(df) == 3 and set(df["schedule"]) == {"GPipe", "1F1B", "Interleaved1F1B"}
    eff = compat.compute_speedup_and_efficiency(df)
    assert len(eff) == 2 and (eff["efficiency"] == eff["speedup"] / 2 * 100).all()
    piv = compat.throughput_pivot(df)
    assert piv.shape == (1, 3)
    compat.plot_speedup_efficiency(eff, str(tmp_path / "eff.png"))
    compat.plot_throughput(df, str(tmp_path / "thr.png"))
    assert os.path.getsize(tmp_path / "eff.png") > 0 and os.path.getsize(tmp_path / "thr.png") > 0
    rep = compat.environment_report()
    assert "torch" in rep and rep["cpu_count"] > 0


def test_native_last_stage_step_returns_merged_logits():
    """schedule.step(target=y, losses=...) on the last rank returns the merged logits
    [B, S, vocab] (reference helper:128, dependency schedules.py:646-652) on the native
    engine too, equal to the reference module's output for the same weights."""
    import torch
    from mipipe.models.ref_transformer import ModelArgs, Transformer, tokenwise_loss_fn
    from mipipe.models.stage import build_reference_stage
    from mipipe.parallel.api import Schedule1F1B
    from mipipe.utils.checkpoint import load_reference_state_dict
    torch.manual_seed(0)
    a = ModelArgs(dim=64, n_layers=2, n_heads=4, vocab_size=100, dim_feedforward=128, dropout=0.0)
    ref = Transformer(a)
    st = build_reference_stage(a, 0, 1, torch.device("cpu"), mbs=2, seq_len=16)
    load_reference_state_dict([st.arena], st.cfg, ref.state_dict())
    sched = Schedule1F1B(st, n_microbatches=4, loss_fn=tokenwise_loss_fn(a.vocab_size))
    x = torch.randint(0, 100, (8, 16))
    y = torch.randint(0, 100, (8, 16))
    losses = []
    out = sched.step(x, target=y, losses=losses)
    assert out.shape == (8, 16, 100) and len(losses) == 4
    torch.testing.assert_close(out.float(), ref(x).detach(), atol=1e-4, rtol=1e-4)
    assert sched.step(x, target=y, losses=[], return_outputs=False) is None


def test_run_train_iterations_reports_bubble():
    m = compat.run_one_experiment(4, 4, 2, "GPipe", batch_size=8, seq_length=16, num_iterations=1, device="cpu",
                                  engine="native", timeout=300)
    assert "error" not in m, m
    assert 0.0 <= m["bubble_fraction"] < 1.0
    assert m["analytic_bubble"] == pytest.approx(1 / 5)


def test_step_outputs_outlive_the_next_step_by_default():
    """the native last stage merges its logits as a view of a persistent buffer
    that the next step rewrites.  Default (reference semantics, torch.cat): a fresh
    tensor, unchanged by later steps; ``copy_outputs=False``: the documented alias."""
    import torch
    from mipipe.models.ref_transformer import ModelArgs, tokenwise_loss_fn
    from mipipe.models.stage import build_reference_stage
    from mipipe.parallel.api import Schedule1F1B
    torch.manual_seed(0)
    a = ModelArgs(dim=64, n_layers=1, n_heads=4, vocab_size=100, dim_feedforward=128, dropout=0.0)
    for copy in (True, False):
        st = build_reference_stage(a, 0, 1, torch.device("cpu"), mbs=2, seq_len=8)
        sched = Schedule1F1B(st, n_microbatches=2, loss_fn=tokenwise_loss_fn(a.vocab_size), copy_outputs=copy)
        x1, x2 = torch.randint(0, 100, (4, 8)), torch.randint(0, 100, (4, 8))
        y = torch.randint(0, 100, (4, 8))
        o1 = sched.step(x1, target=y, losses=[])
        keep = o1.clone()
        o2 = sched.step(x2, target=y, losses=[])
        assert not torch.equal(o2, keep)
        if copy:
            assert torch.equal(o1, keep) and o1.data_ptr() != o2.data_ptr()
        elif o1.data_ptr() == o2.data_ptr():      # the alias: o1 now shows step 2's logits
            assert torch.equal(o1, o2)
