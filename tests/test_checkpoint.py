"""Checkpoint/resume: FQN-keyed per-stage shards + manifest; resuming at a
different pipeline degree (and head mode) continues training exactly like an
uninterrupted run."""
import os

import pytest
import torch

import mipipe  # noqa: F401
from mipipe.engine import PipelineTrainer
from mipipe.models.config import NativeConfig
from mipipe.utils.checkpoint import read_manifest

from dist_utils import run_world

M, MBS, S = 4, 2, 16


def _cfg():
    return NativeConfig.gpt2("tiny", vocab_size=100, d_model=64, n_layers=4, n_heads=4, d_ff=128, max_seq_len=16)


def _data(step):
    g = torch.Generator().manual_seed(100 + step)
    return (torch.randint(0, 100, (M * MBS, S), generator=g), torch.randint(0, 100, (M * MBS, S), generator=g))


def _trainer(pp, split_head=None):
    return PipelineTrainer(_cfg(), pp=pp, schedule="1F1B", n_microbatches=M, mbs=MBS, seq_len=S,
                           device=torch.device("cpu"), dtype=torch.float32, lr=1e-3, split_head=split_head,
                           head_align=8)


def _run(tr, steps, first=0):
    out = []
    for i in range(first, first + steps):
        x, y = _data(i)
        l = tr.train_step(x, y)
        out.append(None if l is None else float(l))
    return out


def _save_worker(rank, world, path, split_head):
    tr = _trainer(world, split_head)
    losses = _run(tr, 2)
    tr.save_checkpoint(path)
    return losses


def _resume_worker(rank, world, path, split_head):
    tr = _trainer(world, split_head)
    man = tr.load_checkpoint(path)
    losses = _run(tr, 2, first=2)
    sd = {k: v.numpy().copy() for k, v in tr.state_dict().items()}
    return dict(losses=losses, sd=sd, step=man["optimizer_step"])


@pytest.mark.parametrize("save_pp,load_pp,save_split,load_split", [(2, 1, False, False), (2, 4, True, True),
                                                                   (4, 2, True, False), (1, 2, False, True)])
def test_resume_resplit_matches_uninterrupted(tmp_path, save_pp, load_pp, save_split, load_split):
    ref = _trainer(1)
    ref_losses = _run(ref, 4)
    ref_sd = ref.state_dict()
    path = str(tmp_path / "ckpt")
    if save_pp == 1:
        _save_worker(0, 1, path, save_split)
    else:
        run_world(_save_worker, save_pp, path, save_split)
    man = read_manifest(path)
    assert man["pp"] == save_pp and man["optimizer_step"] == 2
    assert any(f.startswith("stage-pp") for f in man["shards"])
    if load_pp == 1:
        res = {0: _resume_worker(0, 1, path, load_split)}
    else:
        res = run_world(_resume_worker, load_pp, path, load_split)
    last = res[load_pp - 1]
    assert last["losses"] == pytest.approx(ref_losses[2:], rel=1e-5)
    for r in res.values():
        assert r["step"] == 2
        for k, v in r["sd"].items():
            # Adam normalises tiny fp32 reduction-order differences of near-zero grads
            torch.testing.assert_close(torch.from_numpy(v), ref_sd[k], atol=5e-4, rtol=1e-4)


def test_checkpoint_files_are_fqn_keyed(tmp_path):
    from safetensors import safe_open
    path = str(tmp_path / "c")
    run_world(_save_worker, 2, path, False)
    keys = {}
    for fn in os.listdir(path):
        if fn.startswith("stage-pp"):
            with safe_open(os.path.join(path, fn), framework="pt") as f:
                keys[fn] = set(f.keys())
    assert "tok_embeddings.weight" in keys["stage-pp0.safetensors"]
    assert any(k.startswith("layers.3.") for k in keys["stage-pp1.safetensors"])
    assert "norm.weight" in keys["stage-pp1.safetensors"]
