"""Where the C2 update's batched column-sum finalize (colsum_finalize_batch_kernel, ~20 us per update in r04l) spends
its time: the same segments as one C2 update (K41's 64 slices of the paired hidden dW, the heads' per-block partials,
K42's trunk partials) timed as one flush, then with segments left out, without the clip-norm squares, and the K41
segment alone at other slice counts.

    python tools/finalize_probe.py        # on the GPU box"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main(reps=50):
    import torch
    from xuanpolicy_amd import ops
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    B, K = 65536, 6
    Gh = int(ops.lib().xpa_head_fused_num_partials(B))
    Gt = int(ops.lib().xpa_s3_gemm_trunk_bwd_num_partials(B))

    def seg(G, C):
        return torch.randn(G, C, device=dev, generator=g), torch.empty(C, device=dev)

    k41 = {S: seg(S, 512 * 256) for S in (16, 32, 64)}
    heads = [seg(Gh, C) for C in (K * 256, 256, K, 256, 256, 1)]
    trunk = [seg(Gt, 256 * 17), seg(Gt, 256)]
    sq = torch.zeros(4096, dtype=torch.float64, device=dev)

    def run(segs, use_sq):
        q = ops.ColsumQueue()

        def fn():
            for p, o in segs:
                q.add(p, o)
            q.flush(dev, sq=sq if use_sq else None)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return round(e0.elapsed_time(e1) / reps * 1e3, 2)

    res = {
        "c2_update_segments_sq": run([k41[64]] + heads + trunk, True),
        "c2_update_segments_no_sq": run([k41[64]] + heads + trunk, False),
        "k41_64_alone_sq": run([k41[64]], True),
        "k41_64_alone_no_sq": run([k41[64]], False),
        "k41_32_alone_sq": run([k41[32]], True),
        "k41_16_alone_sq": run([k41[16]], True),
        "heads_trunk_only_sq": run(heads + trunk, True),
        "bytes_k41_64_MiB": 64 * 512 * 256 * 4 / 2 ** 20,
        "note": "event-timed per flush (host launch overhead included when the GPU idles)",
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
