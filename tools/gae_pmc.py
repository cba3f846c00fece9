"""Driver for rocprofv3 --pmc passes over the GAE kernel (K1) at the bench size (4096 x 128) and at
1 M envs, Infinity Cache flushed before every launch.  Run under:
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -- python tools/gae_pmc.py
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d <dir> -- python tools/gae_pmc.py
tools/pmc_summary.py turns the two passes into profiles/pmc_gae_*.json (per-launch HBM bytes of the dense, the
compact and — since r02 — the value-fused form xpa_gae_scan_value, the in-loop launch of the C2 fast path: it also
reads the critic's hidden pre-activations z [2N, 256]; caches evicted by a 512 MiB READ before each of its launches,
so no dirty flush line is written back inside the measured kernel)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from xuanpolicy_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    flush = torch.empty(512 * 1024 * 1024 // 4, device=dev)
    quick = "--quick" in sys.argv   # bench.py's live pass: the bench size (4096 x 128) only
    for N in ((4096,) if quick else (4096, 1048576)):
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
        if N <= 262144:   # value-fused form (z: 2N x 256 f32)
            z = torch.randn(2 * N, 256, device=dev, generator=g)
            w = torch.randn(1, 256, device=dev, generator=g) / 16
            b = torch.zeros(1, device=dev)
            for _ in range(5):
                slot = torch.where(torch.rand(N, device=dev, generator=g) < 0.125,
                                   torch.randint(0, T - 1, (N,), device=dev, generator=g), -1).to(torch.int32)
                flush.sum()
                ops.gae_scan_value(rew, val, term, slot, z, (1, 0.01), w, b, 0.99, 0.95, True, adv=adv, ret=ret,
                                   boot=boot)
            del z
        torch.cuda.synchronize()
        print("N", N, "mid closures", int((closed[:, :-1] > 0).sum()), flush=True)


if __name__ == "__main__":
    main()
