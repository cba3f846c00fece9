"""Driver for rocprofv3 --pmc passes over the GAE kernel (K1) at the bench size (4096 x 128) and at
1 M envs, Infinity Cache flushed before every launch.  Run under:
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -- python tools/gae_pmc.py
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d <dir> -- python tools/gae_pmc.py
tools/pmc_summary.py turns the two passes into profiles/pmc_gae_r01.json (per-launch HBM bytes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from xuanpolicy_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    flush = torch.empty(512 * 1024 * 1024 // 4, device=dev)
    for N in (4096, 1048576):
        T = 128
        g = torch.Generator(device=dev).manual_seed(N)
        rew = torch.randn(N, T, device=dev, generator=g)
        val = torch.randn(N, T, device=dev, generator=g)
        term = (torch.rand(N, T, device=dev, generator=g) < 0.01).float()
        closed = (torch.rand(N, T, device=dev, generator=g) < 0.001).to(torch.uint8)
        closed[:, -1] = 1
        boot = torch.randn(N, T, device=dev, generator=g) * closed
        adv, ret = torch.empty_like(rew), torch.empty_like(rew)
        for _ in range(5):
            flush.fill_(1.0)
            ops.gae_scan(rew, val, term, closed, boot, 0.99, 0.95, True, adv=adv, ret=ret)
        torch.cuda.synchronize()
        print("N", N, "mid closures", int((closed[:, :-1] > 0).sum()), flush=True)


if __name__ == "__main__":
    main()
