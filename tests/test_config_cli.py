"""Config system (YAML/JSON + overrides + reference preset), LR schedule and the
train.py entry point (CPU/gloo, 2 ranks, checkpoint + resume at another PP degree)."""
import json
import os
import subprocess
import sys

import pytest

import mipipe  # noqa: F401
from mipipe.config import RunConfig, TrainSection, lr_at

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("fn", sorted(f for f in os.listdir(os.path.join(ROOT, "configs")) if f.endswith(".yaml")))
def test_shipped_configs_load(fn):
    cfg = RunConfig.load(os.path.join(ROOT, "configs", fn))
    nc = cfg.native_config()
    assert nc.n_layers > 0 and cfg.microbatches >= cfg.parallel.pp


def test_overrides_and_roundtrip(tmp_path):
    cfg = RunConfig.load(os.path.join(ROOT, "configs", "gpt2_small_1f1b_pp4.yaml"),
                         ["parallel.pp=8", "train.lr=1e-3", "model.overrides.n_layers=24", "parallel.split_head=false"])
    assert cfg.parallel.pp == 8 and cfg.train.lr == 1e-3 and cfg.parallel.split_head is False
    assert cfg.native_config().n_layers == 24
    p = str(tmp_path / "c.json")
    cfg.save(p)
    assert RunConfig.load(p).to_dict() == cfg.to_dict()
    with pytest.raises(KeyError):
        cfg.set("train.nope=1")


def test_reference_preset_matches_reference_constants():
    cfg = RunConfig.reference_compat()
    assert cfg.parallel.microbatches == 4 and cfg.train.micro_batch * 4 == 32 and cfg.train.seq_len == 128
    nc = cfg.native_config()
    assert nc.vocab_size == 10000 and nc.d_model == 768 and nc.cross_attn


def test_lr_schedule():
    t = TrainSection(lr=1.0, min_lr=0.1, warmup_steps=10, steps=110)
    assert lr_at(0, t) == pytest.approx(0.1) and lr_at(9, t) == pytest.approx(1.0)
    assert lr_at(10, t) == pytest.approx(1.0) and lr_at(110, t) == pytest.approx(0.1)
    assert lr_at(60, t) == pytest.approx(0.55)


def _torchrun(n, args, port, env=None):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "train.py")] + args
    e = dict(os.environ, OMP_NUM_THREADS="1", **(env or {}))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_train_cli_checkpoint_and_resume_other_pp(tmp_path):
    ck = str(tmp_path / "ck")
    mf = str(tmp_path / "m.jsonl")
    common = ["model.name=gpt2-tiny", "model.overrides.n_layers=4", "model.overrides.d_model=64",
              "model.overrides.n_heads=4", "model.overrides.d_ff=128", "model.overrides.vocab_size=128",
              "train.micro_batch=2", "train.seq_len=32", "train.log_every=1", "train.steps=4",
              f"train.metrics_file={mf}", "parallel.microbatches=4"]
    _torchrun(2, ["--pp", "2"] + common + [f"train.ckpt_dir={ck}", "train.ckpt_every=2"], 29931)
    recs = [json.loads(line) for line in open(mf)]
    assert [r["step"] for r in recs] == [1, 2, 3, 4] and all(r["loss"] > 0 for r in recs)
    assert os.path.exists(os.path.join(ck, "step0000002", "manifest.json"))
    mf2 = str(tmp_path / "m2.jsonl")
    # resume the step-2 checkpoint on ONE rank: steps 3-4 must reproduce the PP=2 run
    out = _torchrun(1, common[:-1] + [f"train.metrics_file={mf2}", "parallel.microbatches=4",
                                      f"train.resume={os.path.join(ck, 'step0000002')}"], 29932)
    assert "resumed" in out
    recs2 = [json.loads(line) for line in open(mf2)]
    assert [r["step"] for r in recs2] == [3, 4]
    for a, b in zip(recs[2:], recs2):
        assert a["loss"] == pytest.approx(b["loss"], rel=1e-4)


def test_watchdog_aborts_hung_step():
    code = ("import sys, time; sys.path.insert(0, %r); import mipipe; "
            "from mipipe.utils.metrics import Watchdog; "
            "wd = Watchdog(1.0, describe=lambda: 'GRID-DUMP'); "
            "ctx = wd.step(); ctx.__enter__(); time.sleep(30)") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 17
    assert "watchdog" in r.stderr and "GRID-DUMP" in r.stderr
