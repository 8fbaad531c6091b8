"""Debug dependency checker and trace ranges: unit checks of the tracker
and a full PP=2 distributed-head training step with MIPIPE_DEBUG=2 (NaN/Inf checks)."""
import pytest
import torch

import mipipe  # noqa: F401
from mipipe.parallel.debug import DependencyError, DepTracker

from dist_utils import run_world


def test_tracker_flags_read_before_wait():
    d = DepTracker(0)
    d.on_post_recv(("F", 1, 0))
    with pytest.raises(DependencyError, match="before its receive completed"):
        d.on_read(("F", 1, 0), "1F0")


def test_tracker_flags_unposted_read_and_double_post():
    d = DepTracker(0)
    with pytest.raises(DependencyError, match="no receive was posted"):
        d.on_read(("B", 0, 3), "0B3")
    d.on_post_recv(("B", 0, 3))
    with pytest.raises(DependencyError, match="posted twice"):
        d.on_post_recv(("B", 0, 3))


def test_tracker_flags_send_before_produce_and_leftovers():
    d = DepTracker(1)
    with pytest.raises(DependencyError, match="before its producer"):
        d.on_send(("F", 2, 0), {})
    d.on_post_recv(("F", 1, 0))
    d.on_wait(("F", 1, 0))
    with pytest.raises(DependencyError, match="never read"):
        d.finish({}, {})
    d2 = DepTracker(1)
    with pytest.raises(DependencyError, match="never sent"):
        d2.finish({("F", 2, 0): None}, {})


def test_tracker_nan_check():
    d = DepTracker(0, level=2)
    with pytest.raises(DependencyError, match="non-finite"):
        d.on_produce(("F", 1, 0), "0F0", (torch.tensor([1.0, float("nan")]),))


def _worker(rank, world):
    from mipipe.engine import PipelineTrainer
    from mipipe.models.config import NativeConfig
    cfg = NativeConfig.gpt2("tiny", vocab_size=100, d_model=64, n_layers=4, n_heads=4, d_ff=128, max_seq_len=16)
    tr = PipelineTrainer(cfg, pp=world, schedule="ZBH1", n_microbatches=4, mbs=2, seq_len=16,
                         device=torch.device("cpu"), dtype=torch.float32, head_align=8)
    assert tr.runtime.deps is not None and tr.runtime.deps.level == 2
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 100, (8, 16), generator=g)
    y = torch.randint(0, 100, (8, 16), generator=g)
    return [float(tr.train_step(x, y)) for _ in range(2)]


def test_full_step_under_dependency_checker(monkeypatch):
    monkeypatch.setenv("MIPIPE_DEBUG", "2")
    monkeypatch.setenv("MIPIPE_RANGES", "1")
    res = run_world(_worker, 2)
    assert res[0] == res[1] and all(l > 0 for l in res[0])
