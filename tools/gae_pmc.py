"""Driver for rocprofv3 --pmc passes over the GAE kernel (K1) at the bench size (4096 x 128) and at
1 M envs, Infinity Cache flushed before every launch.  Run under:
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -- python tools/gae_pmc.py
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d <dir> -- python tools/gae_pmc.py
tools/pmc_summary.py turns the two passes into profiles/pmc_gae_compact_r01.json (per-launch HBM bytes of
the dense and the compact form)."""
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
        vboot = torch.randn(2 * N, device=dev, generator=g)
        for _ in range(5):   # dense form (xpa_gae_scan: closure flags + boot streams)
            flush.fill_(1.0)
            ops.gae_scan(rew, val, term, closed, boot, 0.99, 0.95, True, adv=adv, ret=ret)
        for _ in range(5):   # compact form (the fused agent's in-loop launch), ~1/8 of the rows truncated
            slot = torch.where(torch.rand(N, device=dev, generator=g) < 0.125,
                               torch.randint(0, T - 1, (N,), device=dev, generator=g), -1).to(torch.int32)
            flush.fill_(1.0)
            ops.gae_scan_compact(rew, val, term, slot, vboot, 0.99, 0.95, True, adv=adv, ret=ret, boot=boot)
        torch.cuda.synchronize()
        print("N", N, "mid closures", int((closed[:, :-1] > 0).sum()), flush=True)


if __name__ == "__main__":
    main()
