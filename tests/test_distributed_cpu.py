"""Data-parallel path on CPU with the gloo backend (world_size 2): the flat-gradient all-reduce used per
minibatch (one collective, or an early slice + the rest), parameter broadcast at start-up, and torchrun-style
initialisation."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _net(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(5, 16), torch.nn.LeakyReLU(), torch.nn.Linear(16, 3))


def _data(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(32, 5, generator=g), torch.randn(32, 3, generator=g)


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from xuanpolicy_amd.distributed import GradAllReduce, broadcast_parameters, init_from_env
        from xuanpolicy_amd.flat import FlatState
        r, local, w = init_from_env(backend="gloo")
        assert (r, w) == (rank, world) and dist.get_backend() == "gloo"
        net = _net(seed=rank)           # ranks start different ...
        broadcast_parameters(net)       # ... and leave identical (rank 0's weights)
        ref0 = _net(seed=0)
        for a, b in zip(net.parameters(), ref0.parameters()):
            assert torch.equal(a, b)
        fs = FlatState(net.parameters())
        ar = GradAllReduce(fs)
        assert not ar.early_slice and not ar.begin(fs.params[0].grad)   # default: one collective, no early slice
        ar = GradAllReduce(fs, early_slice=True)
        x, y = _data(rank)
        fs.zero_()
        ((net(x) - y) ** 2).mean().backward()
        ar(fs.params)
        assert ar.calls == 1 and ar.collectives == 1
        # expected: mean over ranks of each rank's local gradient
        exp = []
        for rr in range(world):
            m = _net(seed=0)
            xx, yy = _data(rr)
            ((m(xx) - yy) ** 2).mean().backward()
            exp.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]))
        exp = torch.stack(exp).mean(0)
        got = torch.cat([p.grad.reshape(-1) for p in fs.params])
        torch.testing.assert_close(got, exp, rtol=1e-6, atol=1e-7)
        # the .grad views still alias the (256-B aligned, zero-padded) flat buffer after the collective
        for p, off in zip(fs.params, fs.offsets):
            assert p.grad.data_ptr() == fs.flat[off:].data_ptr() and off % 64 == 0
        assert float(fs.flat.abs().sum()) == float(got.abs().sum())  # padding stays zero
        # early slice (GradAllReduce.begin, as the fused MLP update starts its hidden-pair dW): the same
        # average, element for element, as the single collective
        fs.zero_()
        ((net(x) - y) ** 2).mean().backward()
        whole = fs.flat.clone()
        dist.all_reduce(whole, op=dist.ReduceOp.SUM)
        whole.div_(world)
        w0 = fs.params[2].grad                    # the second Linear's weight: a slice inside the buffer
        c0 = ar.collectives
        assert ar.begin(w0) and not ar.begin(w0)  # one early slice per update
        ar(fs.params)
        assert ar.calls == 2 and ar._early is None and ar.collectives - c0 == 3   # slice inside: 3 calls
        assert torch.equal(fs.flat, whole)
        # a placement group is laid out first: its slice is a prefix, so slice + rest = 2 collectives
        torch.manual_seed(5)
        net2 = torch.nn.Sequential(torch.nn.Linear(5, 16), torch.nn.LeakyReLU(), torch.nn.Linear(16, 4))
        fs2 = FlatState(net2.parameters(), placement=[[net2[2].weight, net2[2].bias]])
        assert fs2.offsets[2] == 0 and fs2.offsets[3] == 64 and fs2.offsets[0] > fs2.offsets[3]
        ar2 = GradAllReduce(fs2, early_slice=True)
        fs2.zero_()
        ((net2(x) - y.repeat(1, 2)[:, :4]) ** 2).mean().backward()
        whole2 = fs2.flat.clone()
        dist.all_reduce(whole2, op=dist.ReduceOp.SUM)
        whole2.div_(world)
        span = fs2.span([net2[2].weight, net2[2].bias])[1]
        assert ar2.begin(span)
        ar2(fs2.params)
        assert ar2.collectives == 2 and torch.equal(fs2.flat, whole2)
        # the learner-level hook (attach_flat_grads + _sync_clip_step, as every minibatch update ends): ONE
        # collective per minibatch by default, and every rank steps to the same parameters
        from xuanpolicy_amd.distributed import attach_flat_grads
        from xuanpolicy_amd.learners import PPOCLIP_Learner
        net3 = _net(seed=0)
        opt = torch.optim.Adam(net3.parameters(), 1e-3, eps=1e-5)

        class _Pol(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.actor = torch.nn.Module()
                self.actor.logstd = torch.nn.Parameter(torch.zeros(1))
                self.body = net3
        pol = _Pol()
        lrn = PPOCLIP_Learner(pol, opt, None, "cpu", "./", 0.25, 0.0, 0.2, 0.5, True)
        attach_flat_grads(lrn, allreduce=True, fused_optimizer=False)
        gs = lrn.grad_sync
        assert gs is not None and not gs.early_slice
        for k in range(3):                        # three minibatches
            xk, yk = _data(rank + 10 * k)
            lrn.flat_grads.zero_()
            ((net3(xk) - yk) ** 2).mean().backward()
            lrn._sync_clip_step()
        assert gs.calls == 3 and gs.collectives == 3, (gs.calls, gs.collectives)
        pv = torch.cat([p.detach().reshape(-1) for p in net3.parameters()])
        allp = [torch.empty_like(pv) for _ in range(world)]
        dist.all_gather(allp, pv)
        assert torch.equal(allp[0], allp[1])
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_flat_grad_allreduce_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=110) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    assert res == {0: "ok", 1: "ok"}, res


def test_init_from_env_single_process_is_noop(monkeypatch):
    from xuanpolicy_amd.distributed import init_from_env
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert init_from_env() == (0, 0, 1)
    assert not dist.is_initialized()
