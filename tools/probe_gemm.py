"""Probe: fp32 GEMM shapes of the PPO update at B=65536 on MI355X (hipBLASLt vs rocBLAS vs manual split-K)."""
import sys
import time

import torch


def bench(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    B = 65536
    shapes = [(256, 256), (6, 256), (1, 256), (256, 17)]  # dW = dY^T [n_out, B] @ X [B, n_in]
    for lib in ("default", "rocblas"):
        if lib == "rocblas":
            torch.backends.cuda.preferred_blas_library("rocblas")
        for (no, ni) in shapes:
            dy = torch.randn(B, no, device=dev)
            x = torch.randn(B, ni, device=dev)
            us = bench(lambda: torch.mm(dy.t(), x))
            fl = 2.0 * B * no * ni
            print(f"{lib:8s} dW [{no}x{ni}] K={B}: {us:8.2f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)
            if lib == "default":
                for S in (8, 16, 32, 64):
                    dys = dy.view(S, B // S, no)
                    xs = x.view(S, B // S, ni)
                    us2 = bench(lambda: torch.bmm(dys.transpose(1, 2), xs).sum(0))
                    print(f"   splitK bmm S={S:3d}: {us2:8.2f} us  {fl / us2 / 1e6:7.1f} TF/s", flush=True)
        torch.backends.cuda.preferred_blas_library("cublaslt" if hasattr(torch.backends.cuda, "preferred_blas_library") else "default")
    # forward / dX shapes for reference
    for (m, k, n) in [(B, 256, 256), (B, 17, 256), (B, 256, 6)]:
        a = torch.randn(m, k, device=dev)
        w = torch.randn(n, k, device=dev)
        us = bench(lambda: torch.nn.functional.linear(a, w))
        print(f"fwd [{m}x{k}]@[{k}x{n}]: {us:8.2f} us {2.0 * m * k * n / us / 1e6:7.1f} TF/s")
    g = torch.randn(B, 256, device=dev)
    us = bench(lambda: g.sum(0))
    print(f"bias grad sum(0) [{B}x256]: {us:.2f} us")


if __name__ == "__main__":
    main()
