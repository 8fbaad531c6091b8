"""The reference's own benchmark workload on ONE MI355X.

BASELINE.md Table 1 times `Transformer(ModelArgs(dim=768, n_layers=L, n_heads=H,
vocab_size=10000))` (post-LN decoder layers with cross-attention over h, ReLU FFN 2048,
dropout 0.1) at batch 32 x seq 128, 4 microbatches, 2 warmup + 5 timed iterations, on a
10-core CPU with gloo (helper:98-143, nb:679-732).  By default (--engine native) this runs the same
model family (native explicit-backward twin, `NativeConfig.reference`) through the
reference-compatible API -- Schedule1F1B.step, the reference's run_train_iterations loop,
fwd+bwd only -- at the reference's precision (f32, on this framework's f32 kernels) at
PP=1 on one GPU, dropout on, and prints one JSON line per (L, H) next to the reference's
best published run for that (L, H) (any P, any schedule) and its GPipe P=2 run.
--engine aten runs the reference's own nn.Module model through the same API (ATen f32);
--engine trainer runs PipelineTrainer (bf16, AdamW included).

Differences, stated: one GPU instead of P CPU processes (the multi-GPU rows need the
8-GPU node the driver owns); timing brackets all work with a device sync.

    python tools/ref_table_gpu.py [--precision fp32|bf16] [--engine native|aten|trainer] [--json out.json]
"""
import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def reference_rows():
    """(L, H, P, schedule) -> tok/s, parsed from BASELINE.md Table 1."""
    rows = {}
    pat = re.compile(r"^\| tokens/s \| (\d+) \| (\d+) \| (\d+) \| (\w+) \| \d+ \| ([\d,\.]+) \|")
    with open(os.path.join(ROOT, "BASELINE.md")) as f:
        for line in f:
            m = pat.match(line)
            if m:
                L, H, P, sched, v = m.groups()
                rows[(int(L), int(H), int(P), sched)] = float(v.replace(",", ""))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--f32-kernels", action="store_true",
                    help="fp32: the linears / attention projections on this framework's f32 MFMA GEMM (gemm_f32.hip) "
                         "instead of ATen (hipBLASLt); 2.3x slower today (profiles/r2_probes.md)")
    ap.add_argument("--precision", default="fp32", choices=["bf16", "fp32"])
    ap.add_argument("--fwd-bwd", action="store_true",
                    help="trainer engine: time the pipeline step alone (forward + backward, no AdamW), the "
                         "reference's timed loop, for a like-for-like comparison with --engine native")
    ap.add_argument("--only", default=None, help="comma list of LxH configs, e.g. 8x8,4x4 (default: all 9)")
    ap.add_argument("--engine", default="native", choices=["native", "aten", "trainer"],
                    help="native: the reference-compatible API (Schedule1F1B over build_reference_stage: this "
                         "framework's kernels at --precision, HIP graphs + native tape + lanes), fwd+bwd only -- "
                         "exactly the reference's timed loop; aten: the reference's own nn.Module model through the "
                         "same API (ATen f32 compute); trainer: PipelineTrainer with the AdamW step (bf16)")
    a = ap.parse_args()
    a.precision_set = "--precision" in sys.argv
    if a.engine == "native":
        return main_native(a)
    if a.engine == "aten":
        return main_fp32(a)
    import torch
    import mipipe  # noqa: F401
    from mipipe.engine import PipelineTrainer
    from mipipe.models.config import NativeConfig

    ref = reference_rows()
    dev = torch.device("cuda", 0)
    B, S, m = 32, 128, 4
    # the trainer's default is bf16; --precision fp32 given explicitly selects f32 arenas
    trainer_dtype = torch.float32 if a.precision_set and a.precision == "fp32" else torch.bfloat16
    out = []
    for L in (4, 8, 12):
        for H in (4, 8, 12):
            if not _selected(a, L, H):
                continue
            cfg = NativeConfig.reference(n_layers=L, n_heads=H)
            tr = PipelineTrainer(cfg, pp=1, schedule="1F1B", n_microbatches=m, mbs=B // m, seq_len=S, device=dev,
                                 seed=0, graphs=not a.no_graphs, dtype=trainer_dtype)
            g = torch.Generator(device="cuda").manual_seed(L * 100 + H)
            x = torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g)
            y = torch.randint(0, cfg.vocab_size, (B, S), device=dev, generator=g)
            if not a.no_graphs:
                tr.capture_graphs(x, y)   # setup (not timed): per-microbatch HIP graphs, dropout-safe
            if a.fwd_bwd:
                ins = [(c,) for c in torch.tensor_split(x, m, dim=0)]
                tgs = list(torch.tensor_split(y, m, dim=0))

                def one():
                    ls = []
                    tr.runtime.step(ins, tgs, ls, return_outputs=False)
                    return torch.stack(ls).mean()
            else:
                def one():
                    return tr.train_step(x, y)
            for _ in range(a.warmup):
                one()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                loss = one()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            tok_s = B * S * a.iters / dt
            mine = {k: v for k, v in ref.items() if k[0] == L and k[1] == H}
            best_k = max(mine, key=mine.get)
            row = {"L": L, "H": H, "tokens_per_s": round(tok_s, 1), "ms_per_iter": round(dt / a.iters * 1e3, 3),
                   "loss": round(float(loss), 4), "lanes": tr.lanes, "ref_best_tok_s": mine[best_k],
                   "ref_best_run": f"P={best_k[2]} {best_k[3]}", "ref_gpipe_p2_tok_s": mine.get((L, H, 2, "GPipe")),
                   "x_vs_ref_best": round(tok_s / mine[best_k], 1)}
            out.append(row)
            print(json.dumps(row), flush=True)
            del tr
            torch.cuda.empty_cache()
    summary = {"config": "reference Transformer(dim 768, vocab 10000, post-LN, cross-attn, ReLU, dropout 0.1), "
                         f"batch 32 x seq 128, m=4, PP=1 on 1 MI355X, {'fp32' if trainer_dtype == torch.float32 else 'bf16'}, "
                         + ("fwd+bwd only, " if a.fwd_bwd else "AdamW step included, ")
                         + ("eager" if a.no_graphs else "HIP graphs") + ", microbatch lanes (MIPIPE_LANES)",
               "rows": out}
    if a.json:
        with open(a.json, "w") as f:
            json.dump(summary, f, indent=1)


def _selected(a, L, H):
    return a.only is None or f"{L}x{H}" in a.only.split(",")


def main_native(a):
    """The reference's workload through the reference-compatible API on this framework's
    kernels: ``native_reference_schedule`` (build_reference_stage at --precision, HIP graphs,
    lanes) + ``run_train_iterations`` (warmup + timed fwd+bwd steps, no optimizer: the
    reference's own loop, helper:98-143) at PP = 1 on one GPU."""
    import torch
    import mipipe  # noqa: F401
    from mipipe.bench.compat import native_reference_schedule, run_train_iterations
    from mipipe.models.ref_transformer import ModelArgs

    ref = reference_rows()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, S, m = 32, 128, 4
    out = []
    for L in (4, 8, 12):
        for H in (4, 8, 12):
            if not _selected(a, L, H):
                continue
            torch.manual_seed(L * 100 + H)
            args = ModelArgs(n_layers=L, n_heads=H)
            sched = native_reference_schedule(args, "1F1B", 0, 1, B, S, m, dev, precision=a.precision)
            x = torch.randint(0, args.vocab_size, (B, S), device=dev)
            y = torch.randint(0, args.vocab_size, (B, S), device=dev)
            met = run_train_iterations(sched, x, y, 0, 1, num_iterations=a.iters, warmup=a.warmup, device=dev,
                                       measure_bubble=False)
            mine = {k: v for k, v in ref.items() if k[0] == L and k[1] == H}
            best_k = max(mine, key=mine.get)
            row = {"L": L, "H": H, "tokens_per_s": round(met["throughput"], 1),
                   "ms_per_iter": round(met["elapsed_time"] / a.iters * 1e3, 3), "precision": met["precision"],
                   "native_runner": met["native_runner"], "lanes": met["lanes"], "ref_best_tok_s": mine[best_k],
                   "ref_best_run": f"P={best_k[2]} {best_k[3]}", "ref_gpipe_p2_tok_s": mine.get((L, H, 2, "GPipe")),
                   "x_vs_ref_best": round(met["throughput"] / mine[best_k], 1)}
            out.append(row)
            print(json.dumps(row), flush=True)
            del sched
            torch.cuda.empty_cache()
    summary = {"config": "reference Transformer(dim 768, vocab 10000, post-LN, cross-attn, ReLU, dropout 0.1), "
                         f"batch 32 x seq 128, m=4, PP=1 on 1 MI355X, {a.precision} on this framework's kernels, "
                         "reference-compatible API (Schedule1F1B.step, merged logits returned), fwd+bwd only "
                         "(no optimizer, helper:98-143), HIP graphs + native tape, microbatch lanes",
               "rows": out}
    if a.json:
        with open(a.json, "w") as f:
            json.dump(summary, f, indent=1)


def main_fp32(a):
    """The reference's workload at the reference's precision: Transformer(ModelArgs(L, H))
    (nn.TransformerDecoderLayer, f32, dropout 0.1) split by manual_model_split into one
    stage, Schedule1F1B(m=4) from mipipe.parallel.api, run_train_iterations' 2 warmup + 5
    timed fwd+bwd steps (no optimizer, as helper:98-143) -- on one MI355X (ATen f32 compute
    through hipBLASLt / MIOpen; the HIP kernels of this framework are bf16-only), with the
    stage replayed as HIP graphs (PipelineStage(graphs=True); --no-graphs: eager)."""
    import torch
    import mipipe  # noqa: F401
    from mipipe.bench.compat import run_train_iterations
    from mipipe.models.ref_transformer import ModelArgs, Transformer, manual_model_split, tokenwise_loss_fn
    from mipipe.parallel.api import Schedule1F1B

    torch.backends.cuda.matmul.allow_tf32 = False
    ref = reference_rows()
    dev = torch.device("cuda", 0)
    B, S, m = 32, 128, 4
    out = []
    for L in (4, 8, 12):
        for H in (4, 8, 12):
            if not _selected(a, L, H):
                continue
            torch.manual_seed(L * 100 + H)
            args = ModelArgs(n_layers=L, n_heads=H)
            stage = manual_model_split(Transformer(args), 0, 1, dev)
            stage.graphs = not a.no_graphs   # one HIP graph per direction and microbatch slot
            stage.f32_kernels = a.f32_kernels   # linears / attention projections on the f32 MFMA GEMM
            sched = Schedule1F1B(stage, n_microbatches=m, loss_fn=tokenwise_loss_fn(args.vocab_size))
            x = torch.randint(0, args.vocab_size, (B, S), device=dev)
            y = torch.randint(0, args.vocab_size, (B, S), device=dev)
            met = run_train_iterations(sched, x, y, 0, 1, num_iterations=a.iters, warmup=a.warmup, device=dev,
                                       measure_bubble=False)
            mine = {k: v for k, v in ref.items() if k[0] == L and k[1] == H}
            best_k = max(mine, key=mine.get)
            row = {"L": L, "H": H, "tokens_per_s": round(met["throughput"], 1),
                   "ms_per_iter": round(met["elapsed_time"] / a.iters * 1e3, 3), "ref_best_tok_s": mine[best_k],
                   "ref_best_run": f"P={best_k[2]} {best_k[3]}", "ref_gpipe_p2_tok_s": mine.get((L, H, 2, "GPipe")),
                   "x_vs_ref_best": round(met["throughput"] / mine[best_k], 1)}
            out.append(row)
            print(json.dumps(row), flush=True)
            del sched, stage
            torch.cuda.empty_cache()
    summary = {"config": "reference Transformer(dim 768, vocab 10000, post-LN, cross-attn, ReLU, dropout 0.1), "
                         "batch 32 x seq 128, m=4, PP=1 on 1 MI355X, **f32** (the reference's precision; ATen "
                         "compute, TF32 off), fwd+bwd only (no optimizer), reference-compatible API, "
                         + ("eager" if a.no_graphs else "HIP graphs per microbatch slot (PipelineStage(graphs=True))")
                         + (", every linear / attention projection on the f32 MFMA GEMM (gemm_f32.hip)"
                            if a.f32_kernels else ", linears on ATen f32"),
               "rows": out}
    if a.json:
        with open(a.json, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
