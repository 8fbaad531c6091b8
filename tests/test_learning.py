"""The engine learns: a model trained on train.py's ``pattern`` stream (every sequence walks
a fixed random permutation, so the next token is a function of the current one) must drive
the loss from ~ln(V) to near zero -- end-to-end evidence that forward, backward, the
pipeline transport, clipping and AdamW are right together (not just that losses match a
reference for one step).  CPU: PP=1 and PP=2 over gloo (distributed head); GPU: HIP graphs
+ native runner + microbatch lanes, GPT-2 and the reference post-LN model with dropout."""
import math
import os
import sys

import pytest
import torch

import mipipe  # noqa: F401
from mipipe.engine import PipelineTrainer
from mipipe.models.config import NativeConfig

from dist_utils import run_world

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import train as _train  # noqa: E402


def _fit(cfg, pp, device, dtype, steps, lr, graphs=False, pattern=48, mbs=8, seq=32, m=2):
    tr = PipelineTrainer(cfg, pp=pp, schedule="1F1B", n_microbatches=m, mbs=mbs, seq_len=seq, device=device,
                         dtype=dtype, lr=lr, seed=0, graphs=graphs)
    data = _train.TokenData(f"pattern:{pattern}", cfg.vocab_size, m * mbs, seq, device, 0, 0)
    if graphs:
        tr.capture_graphs(*data.batch(0))
    losses = []
    for s in range(steps):
        loss = tr.train_step(*data.batch(s))
        if loss is not None:
            losses.append(float(loss))
    return losses


def _tiny(vocab=64):
    return NativeConfig.gpt2("tiny", vocab_size=vocab, d_model=64, n_layers=2, n_heads=4, d_ff=256, max_seq_len=32)


def test_pattern_stream_is_a_permutation_walk():
    d = _train.TokenData("pattern:10", 64, 4, 16, torch.device("cpu"), 0, 3)
    x, y = d.batch(5)
    assert x.max() < 10 and torch.equal(x[:, 1:], y[:, :-1])
    assert torch.equal(d.perm[x], y)
    assert sorted(d.perm.tolist()) == list(range(10))


def test_learns_pattern_pp1_cpu():
    losses = _fit(_tiny(), 1, torch.device("cpu"), torch.float32, 120, 3e-3)
    assert abs(losses[0] - math.log(64)) < 0.5
    assert losses[-1] < 0.05, losses[::20]


def _pp2_worker(rank, world):
    return _fit(_tiny(), 2, torch.device("cpu"), torch.float32, 120, 3e-3)


def test_learns_pattern_pp2_gloo():
    res = run_world(_pp2_worker, 2)
    losses = [l for r in res.values() for l in r]
    assert losses and losses[-1] < 0.05, losses[::20]


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["gpt2", "reference"])
def test_learns_pattern_gpu(model):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mipipe import ops
    assert ops.ext_available()
    dev = torch.device("cuda", 0)
    if model == "gpt2":
        cfg = NativeConfig.gpt2("tiny", vocab_size=512, d_model=256, n_layers=2, n_heads=4, d_ff=1024,
                                max_seq_len=128)
    else:   # post-LN self + cross attention, ReLU, dropout 0.1
        cfg = NativeConfig.reference(n_layers=2, n_heads=4, vocab_size=512, dim=256, dim_feedforward=1024)
    losses = _fit(cfg, 1, dev, torch.bfloat16, 200, 2e-3, graphs=True, pattern=256, mbs=8, seq=128, m=4)
    assert abs(losses[0] - math.log(512)) < 0.7, losses[:3]
    # the median of the last 10 steps: with dropout 0.1 and a constant lr, Adam can spike
    # for a step once the pattern is memorised (the suite's dropout masks depend on the
    # device step counter earlier tests advanced; one run spiked to 4.0 at its very last step)
    tail = sorted(losses[-10:])
    assert all(math.isfinite(x) for x in losses), losses[::20]
    assert tail[len(tail) // 2] < (0.3 if model == "reference" else 0.1), losses[::20]
