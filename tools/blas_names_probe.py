"""Which hipBLASLt kernels does torch pick for the GPT-2 (T = 32768) GEMM shapes?  Run under
rocprofv3 --kernel-trace --stats: the kernel names encode the library's tile config
(MT = macro tile, MIWT = wave tile in MFMA blocks, WG = workgroup shape, PGR / PLR =
prefetch depths, DTL/DTVA = direct-to-LDS).  Also prints per-shape time."""
import torch
import torch.nn.functional as F

T = 32768
SHAPES = {"fwd_qkv": (T, 2304, 768), "fwd_proj": (T, 768, 768), "fwd_fc1": (T, 3072, 768), "fwd_fc2": (T, 768, 3072),
          "dx_qkv": (T, 768, 2304), "dx_fc1": (T, 768, 3072)}


def main():
    torch.manual_seed(0)
    for name, (M, N, K) in SHAPES.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            F.linear(x, w)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            F.linear(x, w)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"{name} {M}x{N}x{K}: {us:.1f} us = {2 * M * N * K / us / 1e6:.0f} TF", flush=True)


if __name__ == "__main__":
    main()
