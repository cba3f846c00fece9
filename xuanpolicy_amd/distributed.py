"""Data-parallel on-policy training across the GPUs of one node (one process per GPU).

The reference has no multi-device path (its only collective, comm.Allreduce in
xuance/common/statistic_tools.py:16, is never enabled).  Here env shards partition across ranks
(each rank owns its own envs, rollout buffer, GAE, permutation and minibatches: no exchange), and the
only collective is ONE all-reduce (average) of the flat fp32 gradient per minibatch, before
clip_grad_norm_, so the clipped norm is the global one.

FlatState (xuanpolicy_amd.flat) makes every parameter's .grad a view into one contiguous buffer, so
autograd accumulates straight into it and the all-reduce is a single RCCL call over xGMI
(latency-bound at 0.04-1 MiB; one bucket, no overlap needed).  Backend "nccl" is RCCL on ROCm; "gloo" is used by the CPU tests.
"""
import os

import torch
import torch.distributed as dist

from .flat import FlatState, FusedClipAdam, fused_adam_compatible


class GradAllReduce:
    """learner.grad_sync hook: average the flat gradient over the process group (one collective)."""

    def __init__(self, flat_grads, group=None):
        self.fg = flat_grads
        self.group = group
        self.world = dist.get_world_size(group)
        self.avg = dist.get_backend(group) == "nccl"
        self.calls = 0

    def __call__(self, params):
        self.fg.ensure_views()
        if self.avg:
            dist.all_reduce(self.fg.flat, op=dist.ReduceOp.AVG, group=self.group)
        else:
            dist.all_reduce(self.fg.flat, op=dist.ReduceOp.SUM, group=self.group)
            self.fg.flat.div_(self.world)
        self.calls += 1


def attach_flat_grads(learner, allreduce=True, group=None, fused_optimizer=True):
    """Give a learner flat parameters/gradients, the fused clip+Adam step when its optimizer allows,
    and the all-reduce hook when a process group of more than one rank is initialised."""
    from .fused_mlp import head_placement
    fs = FlatState(learner.policy.parameters(), placement=head_placement(learner.policy))
    learner.flat_grads = fs
    learner._params = fs.params
    if fused_optimizer and fused_adam_compatible(learner.optimizer):
        learner.fused_opt = FusedClipAdam(learner.optimizer, fs)
    if allreduce and dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        learner.grad_sync = GradAllReduce(fs, group)
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
