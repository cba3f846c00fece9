"""GPU: the data-parallel normalisation variants of SURVEY.md §8(e) with 2 ranks sharing the box's one
GPU over gloo (the RCCL path is the same code with backend "nccl", one GPU per rank):
  * sync_obs_rms   — RMS partials SUM-reduced before the merge == one RunningMeanStd over all ranks' rows;
  * global_advnorm — minibatch advantage moments averaged == adv-norm over the concatenated minibatch;
  * a 2-rank PPO run with both keeps obs statistics and parameters identical on every rank."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), XPA_DIST_BACKEND="gloo")
    import torch.distributed as dist
    try:
        from xuanpolicy_amd import ops
        from xuanpolicy_amd.distributed import init_from_env
        init_from_env()
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        # ---- synchronised RMS ----
        N, D = 300, 17
        xs = [torch.randn(N, D, generator=torch.Generator().manual_seed(10 + r)).to(dev) * (1 + r) + r for r in
              range(world)]
        mean, var = torch.zeros(D, device=dev), torch.ones(D, device=dev)
        count = torch.full((1,), 1e-4, dtype=torch.float64, device=dev)
        for _ in range(3):
            ops.rms_update(xs[rank], mean, var, count,
                           reduce_partials=lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM), world=world)
        m1, v1 = torch.zeros(D, device=dev), torch.ones(D, device=dev)
        c1 = torch.full((1,), 1e-4, dtype=torch.float64, device=dev)
        for _ in range(3):
            ops.rms_update(torch.cat(xs), m1, v1, c1)
        torch.testing.assert_close(mean, m1, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(var, v1, rtol=1e-5, atol=1e-6)
        assert float(count) == float(c1)
        # ---- global adv-norm ----
        B, R, A = 256, 1000, 6
        g = torch.Generator().manual_seed(99)
        adv_all = torch.randn(R, generator=g).to(dev) * 3 + 1
        ret_all = torch.randn(R, generator=g).to(dev)
        act_all = torch.randn(R, A, generator=g).to(dev)
        logp_all = torch.randn(R, generator=g).to(dev) * 0.1 - 5
        idx_all = torch.randperm(R, generator=g)[:B * world].to(dev)
        head_all = torch.randn(B * world, A, generator=g).to(dev) * 0.3
        v_all = torch.randn(B * world, generator=g).to(dev)
        logstd = torch.full((A,), -1.0, device=dev)
        obs_all = torch.randn(R, 3, generator=g).to(dev)
        sl = slice(rank * B, (rank + 1) * B)
        _, part = ops.gather_minibatch(idx_all[sl].contiguous(), obs_all, adv=adv_all)
        dist.all_reduce(part, op=dist.ReduceOp.SUM)
        part.div_(world)
        _, dh, _, _ = ops.policy_loss("ppo", "gaussian", head_all[sl].contiguous(), logstd, v_all[sl].contiguous(),
                                      act_all, adv_all, ret_all, old_logp=logp_all, idx=idx_all[sl].contiguous(),
                                      adv_partials=part)
        dh = dh.clone()
        _, part_c = ops.gather_minibatch(idx_all, obs_all, adv=adv_all)
        _, dh_c, _, _ = ops.policy_loss("ppo", "gaussian", head_all, logstd, v_all, act_all, adv_all, ret_all,
                                        old_logp=logp_all, idx=idx_all, adv_partials=part_c)
        torch.testing.assert_close(dh, dh_c[sl] * world, rtol=1e-5, atol=1e-7)
        # ---- 2-rank PPO with both variants ----
        from xuanpolicy_amd.distributed import broadcast_parameters
        from xuanpolicy_amd.runner import build_synthbox_ppo
        agent = build_synthbox_ppo(n_envs=64, n_steps=16, n_epoch=2, n_minibatch=2, device=dev, shard=rank,
                                   sync_obs_rms=True, global_advnorm=True)
        broadcast_parameters(agent.policy)
        assert agent.sync_obs_rms and agent.global_advnorm and not agent.use_graph
        agent.train(32)
        for t in (agent.obs_mean, agent.obs_var, torch.cat([p.detach().reshape(-1) for p in agent.policy.parameters()])):
            got = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(got, t.contiguous())
            assert torch.equal(got[0], got[1])
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_dp_normalisation_variants_two_ranks_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=580) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res


def _fast_worker(rank, world, port, q):
    """The C2 fast path (hidden [256]: K13 trunk, K14E, K16 heads, split-K dW) on 2 ranks sharing the GPU over
    gloo: ONE all-reduce of the flat gradient per minibatch (north_star), then the same with the opt-in early-slice
    variant (two per minibatch), both leaving every rank with identical parameters."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), XPA_DIST_BACKEND="gloo")
    import torch.distributed as dist
    try:
        from xuanpolicy_amd.distributed import broadcast_parameters, init_from_env
        from xuanpolicy_amd.runner import build_synthbox_ppo
        init_from_env()
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        for early, per_update in ((False, 1), (True, 2)):
            agent = build_synthbox_ppo(n_envs=128, n_steps=16, obs_dim=17, act_dim=6, hidden=256, n_epoch=2,
                                       n_minibatch=2, seed=11, device=dev, shard=rank)
            broadcast_parameters(agent.policy)
            fm = agent.learner._fused_mlp()
            assert fm is not None and fm.gemm_heads and fm.pair is not None, "fast path expected"
            gs = agent.learner.grad_sync
            assert gs is not None and not gs.early_slice
            gs.early_slice = early
            agent.train(32)                     # two iterations of 16 steps, 4 updates each
            torch.cuda.synchronize()
            assert gs.calls == 8 and gs.collectives == 8 * per_update, (early, gs.calls, gs.collectives)
            p = torch.cat([t.detach().reshape(-1) for t in agent.policy.parameters()])
            got = [torch.empty_like(p) for _ in range(world)]
            dist.all_gather(got, p)
            assert torch.equal(got[0], got[1]) and torch.isfinite(p).all()
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_dp_fast_path_one_collective_per_update_two_ranks_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fast_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=580) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res


@pytest.mark.timeout(600)
def test_bench_two_rank_rehearsal_one_gpu():
    """`bench.py --gpus 2` as the driver launches it (torch.distributed.run, one process per rank), both ranks on
    the box's one GPU over gloo: the JSON line reports the whole-job rate of 2 env shards."""
    import json
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, XPA_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(repo, "bench.py"), "--gpus", "2", "--steps",
           "2", "--warmup", "1", "--n-envs", "256", "--horizon", "32", "--n-epoch", "2", "--n-minibatch", "2",
           "--no-sweep", "--no-per", "--no-c3", "--no-c4", "--no-cpu-baseline", "--no-kernel-timing"]
    out = subprocess.run(cmd, cwd=repo, env=env, capture_output=True, text=True, timeout=560)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["steps"] == 2 and r["value"] > 0
    assert r["config"]["global_envs"] == 512 and "dp2" in r["config"]["parallelism"]


@pytest.mark.timeout(900)
def test_bench_self_launch_two_ranks_one_gpu():
    """`python bench.py --gpus 2` with no launcher (the driver's plain form): bench.py starts the 2 ranks itself, both
    on the box's one GPU over gloo, and the line reports n_gpus 2 on the C2 and C4 legs with ONE all-reduce per
    minibatch and the collective's measured time share."""
    import json
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["XPA_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--n-envs", "512", "--horizon", "32", "--n-epoch", "2", "--n-minibatch", "2", "--no-sweep", "--no-per",
           "--no-c1", "--no-c3", "--no-cpu-baseline", "--no-kernel-timing", "--no-pmc", "--no-rocprof"]
    out = subprocess.run(cmd, cwd=repo, env=env, capture_output=True, text=True, timeout=860)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["global_envs"] == 1024 and "dp2" in r["config"]["parallelism"]
    assert r["data_parallel"]["collectives_per_minibatch"] == 1.0
    assert r["data_parallel"]["allreduce"]["bytes"] > 0 and r["data_parallel"]["allreduce_time_share"] > 0
    c4 = r["c4_box376"]
    assert c4["n_gpus"] == 2 and c4["collectives_per_minibatch"] == 1.0 and c4["value"] > 0


def _rollout_sync_worker(rank, world, port, q):
    """sync_obs_rms = "rollout" (r06): the rollout stays graph-captured with the obs-RMS merge folded into K14F, and the
    ranks' statistics are merged once per rollout (agents.rms_rollout_sync): identical obs_rms and parameters on every
    rank after each rollout, with the count = start + every rank's rows."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), XPA_DIST_BACKEND="gloo")
    import torch.distributed as dist
    try:
        from xuanpolicy_amd.distributed import broadcast_parameters, init_from_env
        from xuanpolicy_amd.runner import build_synthbox_ppo
        init_from_env()
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        N, T = 256, 16
        agent = build_synthbox_ppo(n_envs=N, n_steps=T, n_epoch=2, n_minibatch=2, device=dev, shard=rank,
                                   sync_obs_rms="rollout", hidden=256)
        broadcast_parameters(agent.policy)
        assert agent.sync_obs_rms_rollout and not agent.sync_obs_rms and agent.use_graph and agent._k14f_on()
        c_start = float(agent.obs_count)
        agent.train(2 * T)
        torch.cuda.synchronize()
        for t in (agent.obs_mean, agent.obs_var, agent.obs_count,
                  torch.cat([p.detach().reshape(-1) for p in agent.policy.parameters()])):
            got = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(got, t.contiguous())
            assert torch.equal(got[0], got[1])
        # every row merged once: the first observation, then each step's next observation, on every rank
        assert abs(float(agent.obs_count) - (c_start + world * N * (2 * T + 1))) < 1e-3, float(agent.obs_count)
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_sync_obs_rms_per_rollout_two_ranks_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rollout_sync_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=580) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res
