"""Flat parameter / gradient / optimizer-state buffers for the learner's hot path.

Every parameter of the policy becomes a view into one contiguous fp32 buffer, and so does its .grad
(autograd accumulates straight into the views).  That gives:
  * one RCCL all-reduce per minibatch over the whole gradient (xuanpolicy_amd.distributed);
  * one fused clip_grad_norm_ + Adam launch pair over all parameters (xpa_clip_adam_step), replacing
    torch's per-tensor multi_tensor_apply kernels (ppoclip_learner.py:47-49 semantics, see optim.hip).
The torch.optim.Adam object handed in by the runner (runner_drl.py:71) stays the source of truth for
hyper-parameters (lr as stepped by LinearLR, betas, eps) and its .state holds views of the flat moment
buffers, so optimizer.state_dict() / load_state_dict() keep working.
"""
import torch

from . import _lib, ops


ALIGN = 64  # floats: every segment starts on a 256-B boundary (16-B vector kernels on the views)


def _aligned(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


class FlatState:
    """params: the parameters (their order is kept in .params / .offsets).  placement: optional groups
    of parameters laid out back to back in the given order (each member but the last a multiple of
    ALIGN elements), so a group can be used as one tensor — e.g. the actor and critic hidden layers
    that read the same input become one [512, 256] weight (fused_mlp.head_placement)."""

    def __init__(self, params, placement=None):
        self.params = [p for p in params if p.requires_grad]
        index = {id(p): i for i, p in enumerate(self.params)}
        group_of = {}
        for g in placement or []:
            ok = (all(id(p) in index for p in g) and len(set(id(p) for p in g)) == len(g)
                  and all(p.numel() % ALIGN == 0 for p in g[:-1]) and not any(id(p) in group_of for p in g))
            if ok:
                for p in g:
                    group_of[id(p)] = g
        # placement groups first (from offset 0), then the other parameters in order: a group's gradient span
        # is then a prefix of the flat buffer, so an early all-reduce of it plus one of the rest is two
        # collectives per update (distributed.GradAllReduce), never three
        offsets = [None] * len(self.params)
        off = 0
        for g in placement or []:
            if g and id(g[0]) in group_of and group_of[id(g[0])] is g:
                for q in g:
                    offsets[index[id(q)]] = off
                    off += _aligned(q.numel())
        for p in self.params:
            if offsets[index[id(p)]] is None:
                offsets[index[id(p)]] = off
                off += _aligned(p.numel())
        self.offsets = offsets
        n = off
        dev = self.params[0].device
        self.numel = n
        # padding between segments stays zero in param, grad and Adam moments (zero grad -> zero step)
        self.param = torch.zeros(n, dtype=torch.float32, device=dev)
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)  # gradients
        with torch.no_grad():
            for p, off in zip(self.params, self.offsets):
                k = p.numel()
                self.param[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.param[off:off + k].view_as(p)
                p.grad = self.flat[off:off + k].view_as(p)

    def zero_(self):
        self.flat.zero_()

    def span(self, group):
        """(param view, grad view) covering a placement group as one flat span, or None if the members
        are not back to back."""
        offs = []
        for p in group:
            i = next((k for k, q in enumerate(self.params) if q is p), None)
            if i is None:
                return None
            offs.append((self.offsets[i], p.numel()))
        for (o0, n0), (o1, _) in zip(offs, offs[1:]):
            if o1 != o0 + n0:
                return None
        start, total = offs[0][0], sum(n for _, n in offs)
        return self.param[start:start + total], self.flat[start:start + total]

    def ensure_views(self):
        """Re-point .grad at the flat buffer if anything replaced it (e.g. zero_grad(set_to_none=True))."""
        for p, off in zip(self.params, self.offsets):
            k = p.numel()
            view = self.flat[off:off + k]
            if p.grad is None or p.grad.data_ptr() != view.data_ptr():
                g = p.grad
                p.grad = view.view_as(p)
                if g is None:
                    p.grad.zero_()
                else:
                    p.grad.copy_(g)


def fused_adam_compatible(optimizer):
    if type(optimizer) is not torch.optim.Adam or len(optimizer.param_groups) != 1:
        return False
    g = optimizer.param_groups[0]
    return (not g.get("amsgrad", False) and not g.get("maximize", False) and g.get("weight_decay", 0) == 0
            and not g.get("differentiable", False))


class FusedClipAdam:
    """clip_grad_norm_(max_norm) + Adam.step() as two HIP launches over a FlatState."""

    def __init__(self, optimizer, flat: FlatState):
        if not fused_adam_compatible(optimizer):
            raise ValueError("FusedClipAdam needs torch.optim.Adam with one param group, no weight decay/amsgrad")
        group_params = set(id(p) for p in optimizer.param_groups[0]["params"])
        if group_params != set(id(p) for p in flat.params):
            raise ValueError("optimizer parameters differ from the flat state's parameters")
        self.optimizer, self.fs = optimizer, flat
        dev, n = flat.param.device, flat.numel
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.partials = torch.empty(int(ops.lib().xpa_grad_norm_num_partials(n)), dtype=torch.float64, device=dev)
        self.total_norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.step_count = 0
        self._step_t = torch.zeros((), dtype=torch.float32)  # shared CPU 'step' like torch's Adam state
        for p, off in zip(flat.params, flat.offsets):
            k = p.numel()
            st = optimizer.state.get(p, {})
            if "exp_avg" in st:  # migrate existing state
                self.exp_avg[off:off + k].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                self.step_count = int(float(st["step"]))
            optimizer.state[p] = {"step": self._step_t, "exp_avg": self.exp_avg[off:off + k].view_as(p),
                                  "exp_avg_sq": self.exp_avg_sq[off:off + k].view_as(p)}
        self._step_t.fill_(float(self.step_count))

    def step(self, max_norm, sq=None):
        """max_norm: the clip_grad_norm_ bound, or None for no clipping (max_norm = 0 zeroes the gradient,
        as torch's clip_grad_norm_ does).  sq = (float64 partials, count) summing to |grad|^2, written by the
        gradient producers: one launch (xpa_clip_adam_step_partials) instead of the norm pass + step."""
        if max_norm is not None and float(max_norm) < 0:
            raise ValueError("max_norm must be >= 0 (None: no clipping)")
        max_norm = -1.0 if max_norm is None else float(max_norm)   # the kernels' "no clipping" code
        g = self.optimizer.param_groups[0]
        self.step_count += 1
        b1, b2 = g["betas"]
        lr = g["lr"]
        lr = float(lr) if not isinstance(lr, torch.Tensor) else float(lr.item())
        if sq is not None:
            buf, count = sq
            rc = ops.lib().xpa_clip_adam_step_partials(
                ops._p(self.fs.param), ops._p(self.fs.flat), ops._p(self.exp_avg), ops._p(self.exp_avg_sq),
                self.fs.numel, ops._p(buf), int(count), max_norm, lr, float(b1),
                float(b2), float(g["eps"]), self.step_count, ops._p(self.total_norm), ops._stream(self.fs.param.device))
            _lib.check(rc, "xpa_clip_adam_step_partials")
        else:
            rc = ops.lib().xpa_clip_adam_step(ops._p(self.fs.param), ops._p(self.fs.flat), ops._p(self.exp_avg),
                                              ops._p(self.exp_avg_sq), self.fs.numel, ops._p(self.partials),
                                              max_norm, lr, float(b1), float(b2),
                                              float(g["eps"]), self.step_count, ops._p(self.total_norm),
                                              ops._stream(self.fs.param.device))
            _lib.check(rc, "xpa_clip_adam_step")
        self._step_t.fill_(float(self.step_count))
        self.optimizer._opt_called = True  # the LR scheduler checks that an optimizer step happened

    # ---- device schedule: (lr, Adam step) of the next updates in HBM, so K9 can sit inside a captured update ----
    SCHED_WINDOW = 256
    sched_enabled = False

    def enable_sched(self, on=True):
        """Route every step through xpa_clip_adam_step_sched (K9 reading its learning rate and Adam step from a device
        table filled once per SCHED_WINDOW updates): the launch is then graph-capturable."""
        self.sched_enabled = bool(on)
        if on and getattr(self, "_sched", None) is None:
            dev = self.fs.param.device
            self._sched = torch.zeros(2 * self.SCHED_WINDOW, dtype=torch.float32, device=dev)
            self._cursor = torch.zeros(4, dtype=torch.int32, device=dev)
            self._sched_end = self.step_count        # step_count of the last update the table covers
        return self

    def _future_lrs(self, scheduler, count):
        """The learning rates of the next `count` updates: the scheduler stepped ahead on a saved state, then
        restored (its own arithmetic, whatever the schedule)."""
        groups = self.optimizer.param_groups
        g = groups[0]
        if scheduler is None:
            return [float(g["lr"])] * count
        import warnings
        saved_state = scheduler.state_dict()
        saved_lrs = [gg["lr"] for gg in groups]
        saved_called = getattr(self.optimizer, "_opt_called", None)
        out = []
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            for _ in range(count):
                lr = g["lr"]
                out.append(float(lr) if not isinstance(lr, torch.Tensor) else float(lr.item()))
                self.optimizer._opt_called = True
                scheduler.step()
        scheduler.load_state_dict(saved_state)
        for gg, lr in zip(groups, saved_lrs):
            gg["lr"] = lr
        if saved_called is not None:
            self.optimizer._opt_called = saved_called
        return out

    def ensure_window(self, scheduler, need=1):
        """Before `need` updates that launch K9 from the schedule (outside any capture): refill the table and reset the
        cursor unless the current window still covers them.  Stream-ordered H2D copy from a fresh pinned buffer."""
        if need > self.SCHED_WINDOW:
            raise ValueError("%d scheduled updates exceed the %d-entry window" % (need, self.SCHED_WINDOW))
        g = self.optimizer.param_groups[0]
        b1, b2 = g["betas"]
        if self.step_count + need <= self._sched_end and self._window_valid(scheduler, g):
            return
        import ctypes
        import numpy as np
        W = self.SCHED_WINDOW
        lrs = self._future_lrs(scheduler, W)
        # what the table was built from: refilled when any of it changes outside scheduler.step() (a replaced
        # scheduler, an edited param_groups lr, loaded optimizer / scheduler state, other betas)
        self._sched_lrs, self._sched_start = lrs, self.step_count
        self._sched_from = (scheduler, float(b1), float(b2))
        host = torch.zeros(2 * W, dtype=torch.float32).pin_memory()
        out2 = (ctypes.c_float * 2)()
        vals = np.empty(2 * W, dtype=np.float32)
        for k in range(W):
            ops.lib().xpa_adam_sched_entry(lrs[k], float(b1), float(b2), self.step_count + 1 + k,
                                           ctypes.addressof(out2))
            vals[2 * k], vals[2 * k + 1] = out2[0], out2[1]
        host.copy_(torch.from_numpy(vals))
        self._sched.copy_(host, non_blocking=True)
        self._cursor.zero_()
        self._sched_host = host                       # keep the pinned source alive until the copy has run
        self._sched_end = self.step_count + W

    def _window_valid(self, scheduler, g):
        lrs = getattr(self, "_sched_lrs", None)
        if lrs is None:
            return False
        sch, b1, b2 = self._sched_from
        j = self.step_count - self._sched_start
        lr = g["lr"]
        lr = float(lr) if not isinstance(lr, torch.Tensor) else float(lr.item())
        return (sch is scheduler and (b1, b2) == tuple(float(b) for b in g["betas"]) and 0 <= j < len(lrs)
                and lrs[j] == lr)

    def launch_sched(self, max_norm):
        """The device part of a scheduled step (capturable): norm pass + clip + Adam, cursor advanced on device."""
        if max_norm is not None and float(max_norm) < 0:
            raise ValueError("max_norm must be >= 0 (None: no clipping)")
        max_norm = -1.0 if max_norm is None else float(max_norm)
        g = self.optimizer.param_groups[0]
        b1, b2 = g["betas"]
        rc = ops.lib().xpa_clip_adam_step_sched(ops._p(self.fs.param), ops._p(self.fs.flat), ops._p(self.exp_avg),
                                                ops._p(self.exp_avg_sq), self.fs.numel, ops._p(self.partials),
                                                max_norm, float(b1), float(b2), float(g["eps"]), ops._p(self._sched),
                                                self.SCHED_WINDOW, ops._p(self._cursor), ops._p(self.total_norm),
                                                ops._stream(self.fs.param.device))
        _lib.check(rc, "xpa_clip_adam_step_sched")

    def host_step(self):
        """The host bookkeeping of a scheduled step (after its launch or its graph replay)."""
        self.step_count += 1
        self._step_t.fill_(float(self.step_count))
        self.optimizer._opt_called = True

    def sched_overflow(self):
        """True if a scheduled launch ran past its window (host-synchronising read; tests / diagnostics)."""
        return bool(int(self._cursor[2].item()))
