"""Per-launch durations of the same launches by three clocks: dispatch-attached HIP events (hipExtLaunchKernel, the
bench's K1 timer), plain HIP events recorded on the stream around the launch (torch.cuda.Event), and rocprofv3's
kernel trace when run under it.  Empty kernel (xpa_dispatch_floor_timed without events = an empty launch) and the
value-fused GAE scan at C2 after a GEMM (its in-loop predecessor).
    python tools/event_floor.py            (or under rocprofv3 --kernel-trace --output-format csv)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from xuanpolicy_amd import ops  # noqa: E402


def main(reps=30):
    dev = torch.device("cuda:0")
    N, T = 4096, 128
    g = torch.Generator(device=dev).manual_seed(0)
    rew, val = torch.randn(N, T, device=dev, generator=g), torch.randn(N, T, device=dev, generator=g)
    term = (torch.rand(N, T, device=dev, generator=g) < 0.01).float()
    adv, ret, boot = torch.empty_like(rew), torch.empty_like(rew), torch.zeros_like(rew)
    slot = torch.full((N,), -1, dtype=torch.int32, device=dev)
    s_in = torch.randn(2 * N, 256, device=dev, generator=g)
    wh = torch.randn(256, 256, device=dev, generator=g) / 16
    w, b = torch.randn(1, 256, device=dev, generator=g) / 16, torch.zeros(1, device=dev)
    out = {}

    def gae():
        z = torch.nn.functional.linear(s_in, wh)   # the critic GEMM that precedes it in the loop
        return z

    # (b) dispatch-attached events
    ops.TIMER.enabled, ops.TIMER.only = True, {"gae"}
    for i in range(reps + 3):
        z = gae()
        ops.gae_scan_value(rew, val, term, slot, z, (1, 0.01), w, b, 0.99, 0.95, True, adv=adv, ret=ret, boot=boot)
        torch.cuda.synchronize()
        if i == 2:
            ops.TIMER.reset()
    out["gae_dispatch_events_us"] = ops.TIMER.mean_ms("gae") * 1e3
    ops.TIMER.enabled = False
    # (a) stream events around the launch
    ts = []
    for i in range(reps + 3):
        z = gae()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.gae_scan_value(rew, val, term, slot, z, (1, 0.01), w, b, 0.99, 0.95, True, adv=adv, ret=ret, boot=boot)
        e1.record()
        e1.synchronize()
        if i >= 3:
            ts.append(e0.elapsed_time(e1) * 1e3)
    out["gae_stream_events_us"] = sum(ts) / len(ts)
    # empty launch: both clocks
    out["empty_dispatch_events_us"] = ops.dispatch_floor_us(dev, reps)
    st = ops._stream(dev)
    ts = []
    for i in range(reps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.lib().xpa_dispatch_floor_timed(None, None, st)
        e1.record()
        e1.synchronize()
        if i >= 3:
            ts.append(e0.elapsed_time(e1) * 1e3)
    out["empty_stream_events_us"] = sum(ts) / len(ts)
    print(json.dumps({k: round(v, 3) for k, v in out.items()}))


if __name__ == "__main__":
    main()
