"""CPU/gloo multi-process plumbing tests (SURVEY §4 tier 2, BASELINE config 1).

Pipelined gradients and losses must equal a single-process, non-pipelined run of
the same reference Transformer (dropout 0, same seed)."""
import pytest
import torch

import mipipe  # noqa: F401
from mipipe.models.ref_transformer import ModelArgs, Transformer, manual_model_split, tokenwise_loss_fn
from mipipe.parallel.api import get_schedule_class

from dist_utils import run_world

ARGS = dict(dim=32, n_layers=4, n_heads=4, vocab_size=50, dim_feedforward=64, dropout=0.0)
B, S, M = 8, 6, 4


def _data():
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, ARGS["vocab_size"], (B, S), generator=g)
    y = torch.randint(0, ARGS["vocab_size"], (B, S), generator=g)
    return x, y


def _reference_grads():
    torch.manual_seed(0)
    model = Transformer(ModelArgs(**ARGS))
    x, y = _data()
    loss_fn = tokenwise_loss_fn(ARGS["vocab_size"])
    losses = []
    for xc, yc in zip(torch.tensor_split(x, M), torch.tensor_split(y, M)):
        loss = loss_fn(model(xc), yc)
        losses.append(loss.item())
        (loss / M).backward()
    return {n: p.grad.clone() for n, p in model.named_parameters()}, losses


def _worker(rank, world, sched, v):
    import torch
    import torch.distributed as dist
    x, y = _data()
    num_stages = world * v
    stages = []
    for i in range(v):
        torch.manual_seed(0)
        model = Transformer(ModelArgs(**ARGS))
        stages.append(manual_model_split(model, rank + world * i, num_stages, torch.device("cpu")))
    cls = get_schedule_class(sched)
    schedule = cls(stages if v > 1 else stages[0], n_microbatches=M, loss_fn=tokenwise_loss_fn(ARGS["vocab_size"]))
    losses = []
    out = None
    for _ in range(1):
        if rank == 0 and rank == world - 1:
            out = schedule.step(x, target=y, losses=losses)
        elif rank == 0:
            schedule.step(x)
        elif rank == world - 1:
            out = schedule.step(target=y, losses=losses)
        else:
            schedule.step()
    grads = {}
    for st in stages:
        for n, p in st.submod.named_parameters():
            grads[n] = p.grad.numpy().copy()  # numpy: no shared-memory fds across exit
    return dict(grads=grads, losses=[l.item() for l in losses], out_shape=None if out is None else tuple(out.shape))


@pytest.mark.parametrize("sched,world,v", [("GPipe", 2, 1), ("1F1B", 2, 1), ("1F1B", 4, 1),
                                           ("Interleaved1F1B", 2, 2), ("LoopedBFS", 2, 2), ("ZBH1", 2, 1)])
def test_pipeline_grads_match_single_process(sched, world, v):
    ref_grads, ref_losses = _reference_grads()
    res = run_world(_worker, world, sched, v)
    got = {}
    for r in res.values():
        got.update({k: torch.from_numpy(v) for k, v in r["grads"].items()})
    assert set(got) == set(ref_grads), "stage state_dicts must keep global FQNs"
    for n, g in ref_grads.items():
        torch.testing.assert_close(got[n], g, rtol=1e-4, atol=1e-5, msg=lambda m: f"{n}: {m}")
    last = res[world - 1]
    assert last["losses"] == pytest.approx(ref_losses, rel=1e-5)
    assert last["out_shape"] == (B, S, ARGS["vocab_size"])


def test_single_rank_pipeline_no_dist():
    """PP=1 (no process group): the schedule degenerates to gradient accumulation."""
    ref_grads, ref_losses = _reference_grads()
    torch.manual_seed(0)
    model = Transformer(ModelArgs(**ARGS))
    stage = manual_model_split(model, 0, 1, torch.device("cpu"))
    x, y = _data()
    losses = []
    sched = get_schedule_class("1F1B")(stage, n_microbatches=M, loss_fn=tokenwise_loss_fn(ARGS["vocab_size"]))
    sched.step(x, target=y, losses=losses)
    for n, p in stage.submod.named_parameters():
        torch.testing.assert_close(p.grad, ref_grads[n], rtol=1e-4, atol=1e-5)
    assert [l.item() for l in losses] == pytest.approx(ref_losses, rel=1e-5)
