"""CPU: sync_obs_rms = "rollout" (r06, agents.rms_rollout_sync) — every rank's rollout rows recovered from its running
statistics (start (+) rows, merged step by step with f32 storage as the device does) and merged across ranks into the
common start statistics equal one RunningMeanStd (statistic_tools.py:86-112, f64) over the start rows and every rank's
rows, within the f32 storage's rounding.  The all-reduce is simulated in-process (a SUM over the ranks' vectors)."""
import numpy as np
import torch

from xuanpolicy_amd.agents import rms_rollout_sync


def _merge(mean, var, count, x):
    """RunningMeanStd.update on the batch x (f64 arithmetic), then the f32 storage of mean / var (the device's)."""
    bm, bv, n = x.mean(0), x.var(0), x.shape[0]
    tot = count + n
    delta = bm - mean
    new_mean = mean + delta * n / tot
    new_var = (var * count + bv * n + delta ** 2 * count * n / tot) / tot
    return new_mean.astype(np.float32).astype(np.float64), new_var.astype(np.float32).astype(np.float64), tot


def test_rollout_sync_equals_one_rms_over_all_rows():
    rng = np.random.default_rng(0)
    D, R, steps, N = 17, 4, 16, 64
    x0 = rng.normal(1.0, 2.0, (3 * N, D))
    m, v, c = np.zeros(D), np.ones(D), 1e-4
    for k in range(3):
        m, v, c = _merge(m, v, c, x0[k * N:(k + 1) * N])
    start = (torch.tensor(m, dtype=torch.float32), torch.tensor(v, dtype=torch.float32),
             torch.tensor([c], dtype=torch.float64))
    rows = [rng.normal(0.5 * r, 1.0 + r, (steps * N, D)) for r in range(R)]
    ends = []
    for r in range(R):
        mr, vr, cr = m, v, c
        for k in range(steps):
            mr, vr, cr = _merge(mr, vr, cr, rows[r][k * N:(k + 1) * N])
        ends.append((torch.tensor(mr, dtype=torch.float32), torch.tensor(vr, dtype=torch.float32),
                     torch.tensor([cr], dtype=torch.float64)))
    reds = []
    for r in range(R):   # pass 1: each rank's contribution
        rms_rollout_sync(start, ends[r], lambda t: reds.append(t.clone()))
    total = torch.stack(reds).sum(0)
    outs = []
    for r in range(R):   # pass 2: the all-reduce's result on every rank

        def ar(t):
            t.copy_(total)
        outs.append(rms_rollout_sync(start, ends[r], ar))
    for o in outs[1:]:   # every rank leaves with the same statistics
        assert all(torch.equal(a, b) for a, b in zip(o, outs[0]))
    allx = np.concatenate([x0] + rows)
    cnt = 1e-4 + allx.shape[0]
    bm, bv = allx.mean(0), allx.var(0)
    ref_mean = bm * allx.shape[0] / cnt
    ref_var = (1.0 * 1e-4 + bv * allx.shape[0] + bm ** 2 * 1e-4 * allx.shape[0] / cnt) / cnt
    mean, var, count = outs[0]
    assert abs(float(count) - cnt) < 1e-6
    np.testing.assert_allclose(mean.numpy(), ref_mean, rtol=2e-5, atol=2e-6)
    np.testing.assert_allclose(var.numpy(), ref_var, rtol=2e-5, atol=2e-6)
