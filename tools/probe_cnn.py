"""Probe MIOpen algorithm / layout choices for the C3 AC_CNN_Atari update (B = 16 384 frames).

    python tools/probe_cnn.py
Times forward + backward of the trunk (conv 8/4 -> 4/2 -> 3/1 -> fc 512, ReLU) + a linear head for
  layout nhwc  : the reference's permute(0, 3, 1, 2) view of the uint8 NHWC frames (channels-last)
  layout nchw  : frames converted to a contiguous NCHW float tensor first
with torch.backends.cudnn.benchmark (MIOpen exhaustive find) off and on."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from xuanpolicy_amd.policies import AC_CNN_Atari
    dev = torch.device("cuda:0")
    B = 16384
    frames = torch.randint(0, 256, (B, 84, 84, 4), device=dev, dtype=torch.int32).to(torch.uint8)
    res = {}
    for bench in (False, True):
        torch.backends.cudnn.benchmark = bench
        for layout in ("nhwc", "nchw"):
            torch.manual_seed(0)
            rep = AC_CNN_Atari((84, 84, 4), [8, 4, 3], [4, 2, 1], [32, 64, 64], None, None, torch.nn.ReLU, dev, [512])
            head = torch.nn.Linear(512, 7).to(dev)
            params = list(rep.parameters()) + list(head.parameters())

            def step():
                x = frames.float() / 255.0
                x = x.permute(0, 3, 1, 2)
                if layout == "nchw":
                    x = x.contiguous()
                out = head(rep.model(x))
                loss = out.square().mean()
                grads = torch.autograd.grad(loss, params)
                return grads
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            t = time.perf_counter()
            n = 5
            for _ in range(n):
                step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / n * 1e3
            res[(bench, layout)] = ms
            print("benchmark=%s layout=%s: %.2f ms per fwd+bwd (B=%d)" % (bench, layout, ms, B), flush=True)
    return res


if __name__ == "__main__":
    main()
