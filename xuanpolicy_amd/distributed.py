"""Data-parallel on-policy training across the GPUs of one node (one process per GPU).

The reference has no multi-device path (its only collective, comm.Allreduce in
xuance/common/statistic_tools.py:16, is never enabled).  Here env shards partition across ranks
(each rank owns its own envs, rollout buffer, GAE, permutation and minibatches: no exchange), and the
only collective is ONE all-reduce (average) of the flat fp32 gradient per minibatch, before
clip_grad_norm_, so the clipped norm is the global one.

FlatState (xuanpolicy_amd.flat) makes every parameter's .grad a view into one contiguous buffer, so
autograd accumulates straight into it and the all-reduce is one RCCL call over xGMI per minibatch
(latency-bound at 0.04-1 MiB; one bucket).  That single collective is the default (north_star: "a single
RCCL all-reduce of gradients per minibatch").  GradAllReduce(early_slice=True) is an opt-in variant for the
fused MLP path that issues two: the paired hidden layers' dW slice (the first 0.5 MB of the flat buffer) is
started as soon as its GEMM has written it and overlaps the rest of the backward (GradAllReduce.begin), the
rest is one more call.  That overlap is exercised with gloo only; no RCCL measurement justifies it yet, so it
stays off.  Backend "nccl" is RCCL on ROCm; "gloo" is used by the CPU tests.
"""
import os

import torch
import torch.distributed as dist

from .flat import FlatState, FusedClipAdam, fused_adam_compatible


class GradAllReduce:
    """learner.grad_sync hook: average the flat gradient over the process group.

    begin(region): start the all-reduce of one contiguous slice of the flat gradient early (async, on the
    collective's own stream) as soon as its producer has written it — the fused MLP update hands over the
    paired hidden layers' dW (0.5 MB of C2's 0.55 MB) right after its GEMM, so the transfer overlaps the dX
    GEMM and the trunk backward.  __call__ then reduces the rest of the buffer and waits for the early
    slice: every element is still averaged exactly once, before the clip."""

    def __init__(self, flat_grads, group=None, early_slice=False):
        self.fg = flat_grads
        self.early_slice = bool(early_slice)
        self.group = group
        self.world = dist.get_world_size(group)
        self.avg = dist.get_backend(group) == "nccl"
        self.calls = 0
        self.collectives = 0  # all_reduce calls issued: 1 per minibatch (2 with early_slice on the fused MLP path)
        self._early = None   # (offset, numel, work)

    def _reduce(self, t, async_op=False):
        op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
        self.collectives += 1
        return dist.all_reduce(t, op=op, group=self.group, async_op=async_op)

    def begin(self, region):
        """Start the async all-reduce of `region` (a contiguous view into the flat gradient).  Returns False (and
        does nothing) unless early_slice is on."""
        if not self.early_slice:
            return False
        flat = self.fg.flat
        off = (region.data_ptr() - flat.data_ptr()) // flat.element_size()
        n = region.numel()
        if (self._early is not None or not region.is_contiguous() or off < 0 or off + n > flat.numel()
                or region.dtype != flat.dtype):
            return False
        self._early = (off, n, self._reduce(flat[off:off + n], async_op=True))
        return True

    def __call__(self, params):
        self.fg.ensure_views()
        flat = self.fg.flat
        if self._early is None:
            self._reduce(flat)
            if not self.avg:
                flat.div_(self.world)
        else:
            off, n, work = self._early
            self._early = None
            # FlatState lays the paired hidden layers out first, so the early slice is a prefix and the rest
            # is ONE range; a slice elsewhere costs one more collective for the range before it
            for lo, hi in ((0, off), (off + n, flat.numel())):
                if hi > lo:
                    self._reduce(flat[lo:hi])
            work.wait()   # NCCL: the current stream waits for the early slice (no host sync)
            if not self.avg:
                flat.div_(self.world)
        self.calls += 1


class LocalGradSync:
    """A world-size-1 stand-in for GradAllReduce (no collective): attached to a learner on one GPU it makes the update
    take exactly the data-parallel code path — the clip norm from its own pass over the (synchronised) flat gradient
    instead of the producers' partials, eager K9 instead of the device-scheduled / graphed step — so that path's
    per-rank cost is measurable before a multi-GPU node exists (bench.py --dp-path)."""

    early_slice = False

    def __init__(self, flat_grads):
        self.fg = flat_grads
        self.avg = True
        self.calls = 0
        self.collectives = 0

    def begin(self, region):
        return False

    def __call__(self, params):
        self.fg.ensure_views()
        self.calls += 1


def attach_flat_grads(learner, allreduce=True, group=None, fused_optimizer=True, early_slice=False):
    """Give a learner flat parameters/gradients, the fused clip+Adam step when its optimizer allows,
    and the all-reduce hook when a process group of more than one rank is initialised (one collective per
    minibatch; early_slice=True: the two-collective overlapped variant)."""
    from .fused_mlp import head_placement
    fs = FlatState(learner.policy.parameters(), placement=head_placement(learner.policy))
    learner.flat_grads = fs
    learner._params = fs.params
    if fused_optimizer and fused_adam_compatible(learner.optimizer):
        learner.fused_opt = FusedClipAdam(learner.optimizer, fs)
    if allreduce and dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        learner.grad_sync = GradAllReduce(fs, group, early_slice=early_slice)
    return fs


def broadcast_parameters(module, src=0, group=None):
    """Start every rank from rank src's weights (one broadcast per tensor, at setup only)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        with torch.no_grad():
            for t in list(module.parameters()) + list(module.buffers()):
                dist.broadcast(t, src, group=group)


def init_from_env(backend=None):
    """torchrun-style init (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        backend = backend or os.environ.get("XPA_DIST_BACKEND")  # e.g. gloo for a 1-GPU rehearsal
        if backend is None:
            backend = "nccl" if torch.cuda.device_count() > 0 else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, local, world


def local_device(local_rank):
    """cuda:<local_rank>, wrapped onto the visible devices (several ranks may share one GPU in a
    gloo rehearsal; with RCCL every rank has its own GPU)."""
    n = torch.cuda.device_count()
    return torch.device("cuda", local_rank % n) if n else torch.device("cpu")
