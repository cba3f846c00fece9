"""Probe: weight-gradient GEMMs with a tiny output dim at K = 65 536 (split count / orientation)."""
import torch

from probe_gemm import bench


def main():
    dev = torch.device("cuda:0")
    B = 65536
    for (no, ni) in [(6, 256), (1, 256), (256, 17), (17, 256)]:
        dz = torch.randn(B, no, device=dev)
        x = torch.randn(B, ni, device=dev)
        out = torch.empty(no, ni, device=dev)
        outT = torch.empty(ni, no, device=dev)
        res = []
        for s in (1, 8, 16, 32, 64, 128, 256):
            a = dz.view(s, B // s, no)
            b = x.view(s, B // s, ni)
            us = bench(lambda: torch.sum(torch.bmm(a.transpose(1, 2), b), 0, out=out))
            usT = bench(lambda: torch.sum(torch.bmm(b.transpose(1, 2), a), 0, out=outT))
            res.append((s, round(us, 1), round(usT, 1)))
        print(f"dW [{no}x{ni}] (S, us dz^T x, us x^T dz):", res, flush=True)


if __name__ == "__main__":
    main()
