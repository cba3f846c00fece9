"""PPO-Clip and A2C learners whose loss forward+backward runs in hand-written HIP kernels (K2 / K12).

Mirrors (reference paths):
  Learner               xuance/torch/learners/learner.py:10-52 (save_model / load_model / update)
  PPOCLIP_Learner       xuance/torch/learners/policy_gradient/ppoclip_learner.py:4-65
  A2C_Learner           xuance/torch/learners/policy_gradient/a2c_learner.py:4-50
Same constructor arguments, same update() signature and the same info-dict keys.

Per update (reference order, ppoclip_learner.py:45-51): forward, loss, backward -> [one flat gradient
all-reduce when data-parallel] -> clip_grad_norm_ -> optimizer.step -> scheduler.step.
  * update(): policy heads forward (PyTorch-ROCm GEMMs) -> K2 xpa_policy_loss_fwd_bwd + finalize
    (loss scalars, d loss/d mu|logits, d loss/d logstd, d loss/d v) -> autograd backward of those
    head gradients -> K9 fused clip + Adam when the parameters are flat.
  * update_fused() (the agent's hot loop, MLP policies with flat parameters): fused_mlp's explicit
    forward/backward with K13 (first layer), one paired hidden GEMM, K12 (heads + loss + head
    backward) and K9 — no autograd graph.  update() returns host floats like the reference (one sync);
update_fused() keeps everything on device for the agent's hot loop.
"""
import ctypes
import os

import torch

from . import _lib, ops
from .policies import policy_discrete, policy_heads


class Learner:
    def __init__(self, policy, optimizer, scheduler=None, device=None, model_dir="./"):
        self.policy = policy
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.device = device
        self.model_dir = model_dir
        self.iterations = 0
        self.grad_sync = None  # set by xuanpolicy_amd.distributed for data-parallel training

    def save_model(self, model_path):
        torch.save(self.policy.state_dict(), model_path)

    def load_model(self, path, seed=1):
        """learner.py:27-48: newest file of the seed_<seed> directory."""
        for f in os.listdir(path):
            if "seed_%d" % seed in f:
                path = os.path.join(path, f)
                break
        names = sorted(n for n in os.listdir(path) if n != "obs_rms.npy")
        dev = self.device if self.device is not None else "cpu"
        self.policy.load_state_dict(torch.load(os.path.join(path, names[-1]), map_location=dev, weights_only=True))
        fc = getattr(self, "_fc", None)
        if fc:
            fc.stale = True

    def update(self, *args):
        raise NotImplementedError


def _dist_of(policy):
    return "categorical" if policy_discrete(policy) else "gaussian"


class _FusedPolicyGradient(Learner):
    algo = "ppo"

    def __init__(self, policy, optimizer, scheduler, device, model_dir, vf_coef, ent_coef, clip_range, max_grad_norm,
                 use_grad_clip):
        super().__init__(policy, optimizer, scheduler, device, model_dir)
        self.vf_coef, self.ent_coef, self.clip_range = vf_coef, ent_coef, clip_range
        self._max_norm, self._use_clip = max_grad_norm, use_grad_clip
        self.dist = _dist_of(policy)
        self._ws = None
        self._params = [p for p in policy.parameters()]

    def _backward_and_step(self, head, logstd, v, d_head, d_logstd, d_v):
        fg = getattr(self, "flat_grads", None)
        if fg is not None:
            fg.zero_()  # grads are views into one flat buffer (xuanpolicy_amd.distributed.FlatGrads)
        else:
            self.optimizer.zero_grad(set_to_none=True)
        tensors, grads = [head, v], [d_head, d_v]
        if logstd is not None:
            tensors.append(logstd)
            grads.append(d_logstd)
        torch.autograd.backward(tensors, grads)
        self._sync_clip_step()

    def _fused_mlp(self):
        """Explicit actor-critic backward (fused_mlp.FusedActorCritic) once gradients live in flat views."""
        fm = getattr(self, "_fm", None)
        if fm is None and getattr(self, "flat_grads", None) is not None and getattr(self, "fused_mlp_enabled", True):
            from .fused_mlp import FusedActorCritic
            try:
                fm = FusedActorCritic(self.policy, flat=self.flat_grads)
            except ValueError:
                fm = False
            self._fm = fm
        return fm or None

    def _fused_cnn(self):
        """Explicit CNN actor-critic forward/backward (fused_cnn.FusedCNNActorCritic) for AC_CNN_Atari policies."""
        fc = getattr(self, "_fc", None)
        if fc is None:
            fc = False
            if getattr(self, "fused_cnn_enabled", True) and self._device().type == "cuda":
                from .fused_cnn import FusedCNNActorCritic
                try:
                    fc = FusedCNNActorCritic(self.policy)
                except ValueError:
                    fc = False
            self._fc = fc
        return fc or None

    def _sync_clip_step(self, sq=None):
        """sq = (partials, count): squared-norm partials of the complete gradient written by its producers
        (valid only without a gradient all-reduce): the fused step skips its norm pass."""
        if self.grad_sync is not None:
            self.grad_sync(self._params)
            sq = None
        fused = getattr(self, "fused_opt", None)
        if fused is not None and fused.sched_enabled and self.grad_sync is None:
            fused.ensure_window(self.scheduler)
            fused.launch_sched(self._max_norm if self._use_clip else None)   # K9 from the device schedule
            fused.host_step()
        elif fused is not None:
            fused.step(self._max_norm if self._use_clip else None, sq=sq)  # xpa_clip_adam_step (K9)
        else:
            if self._use_clip:
                torch.nn.utils.clip_grad_norm_(self._params, self._max_norm)
            self.optimizer.step()
        if self.scheduler is not None:
            self.scheduler.step()

    def update_fused(self, obs, idx, act, adv, ret, old_logp=None, adv_partials=None, pre=None):
        """One minibatch update reading act/adv/ret/old_logp from the flattened rollout buffer at idx
        (idx=None: already gathered).  pre: launches that produce obs / adv_partials (the agent's minibatch gather),
        run first — inside the slot graph when the update is graphed.  Returns the device tensor of loss scalars
        (ops.OUT_KEYS)."""
        self.iterations += 1
        if pre is not None and not (self._fused_mlp() is not None and not self._fused_mlp().fused_heads
                                    and self._graph_ok(obs)):
            pre()
            pre = None
        fm = self._fused_mlp()
        if fm is not None and fm.fused_heads:
            fm.early_grad_sync = (self.grad_sync.begin if getattr(self.grad_sync, "early_slice", False) else None)
            # obs may be fused_mlp.Rows(flat buffer, idx): K13 reads the minibatch through idx and, with adv_partials,
            # writes the minibatch's advantage moments itself (no K4 launch)
            rows = type(obs).__name__ == "Rows"
            ctx = fm.forward_hidden(obs, adv=adv if rows else None, adv_partials=adv_partials if rows else None)
            scalars = fm.loss_backward(ctx, self.algo, self.dist, act, adv, ret, old_logp=old_logp, idx=idx,
                                       adv_partials=adv_partials, clip_range=self.clip_range, vf_coef=self.vf_coef,
                                       ent_coef=self.ent_coef)
            self._sync_clip_step(sq=fm.sq_ready)
            return scalars
        fc = self._fused_cnn() if fm is None else None
        if fc is not None and obs.dtype == torch.uint8:
            # explicit CNN path: K20 frames, MIOpen convs + K21 bias/ReLU, K2 loss, K22 + conv/GEMM backward
            head, logstd, v, ctx = fc.forward(obs)
            if self._ws is None or self._ws.batch != head.shape[0]:
                self._ws = ops.LossWorkspace(head.shape[0], head.shape[1], head.device, self.dist)
            fg = getattr(self, "flat_grads", None)
            if fg is None:
                for p in self._params:
                    if p.grad is None:
                        p.grad = torch.zeros_like(p)
            scalars, dh, _, dv = ops.policy_loss(self.algo, self.dist, head, logstd, v.contiguous(), act, adv, ret,
                                                 old_logp=old_logp, idx=idx, adv_partials=adv_partials,
                                                 clip_range=self.clip_range, vf_coef=self.vf_coef,
                                                 ent_coef=self.ent_coef, ws=self._ws,
                                                 d_logstd_out=logstd.grad if logstd is not None else None)
            fc.backward(ctx, dh, dv)       # writes every parameter gradient
            self._sync_clip_step()
            return scalars
        if fm is not None and self._graph_ok(obs):
            fused = getattr(self, "fused_opt", None)
            if fused is not None and getattr(self, "graph_k9", True):
                # K9 inside the slot graph: it reads lr / Adam step from the device schedule and advances its cursor
                if not fused.sched_enabled:
                    fused.enable_sched()
                fused.ensure_window(self.scheduler)
                scalars = self._graphed_mlp_update(fm, obs, idx, act, adv, ret, old_logp, adv_partials, pre,
                                                   k9=lambda: fused.launch_sched(self._max_norm if self._use_clip
                                                                                 else None))
                fused.host_step()
                if self.scheduler is not None:
                    self.scheduler.step()
                return scalars
            scalars = self._graphed_mlp_update(fm, obs, idx, act, adv, ret, old_logp, adv_partials, pre)
            self._sync_clip_step()
            return scalars
        if fm is not None:
            return self._mlp_update(fm, obs, idx, act, adv, ret, old_logp, adv_partials, step=True)
        head, logstd, v = policy_heads(self.policy, obs)
        if self._ws is None or self._ws.batch != head.shape[0]:
            self._ws = ops.LossWorkspace(head.shape[0], head.shape[1], head.device, self.dist)
        scalars, dh, dls, dv = ops.policy_loss(self.algo, self.dist, head.contiguous(), logstd, v.contiguous(), act, adv,
                                               ret, old_logp=old_logp, idx=idx, adv_partials=adv_partials,
                                               clip_range=self.clip_range, vf_coef=self.vf_coef,
                                               ent_coef=self.ent_coef, ws=self._ws)
        self._backward_and_step(head, logstd, v, dh, dls, dv)
        return scalars

    # Small minibatches (C1: 128 rows of a [64] net) are bound by host dispatch, ~20 launches of a few us each at
    # ~15-20 us of host time apiece (profiles/r02f_c1_host_probe.txt).  The explicit forward + loss + backward of one
    # minibatch slot is therefore captured once into a hipGraph and replayed.  Every input is a fixed buffer: the rollout
    # columns, the persistent epoch permutation (idx is a slice of it) and the gathered obs rows.  The parameters are
    # updated in place by K9, which is captured too (r03): it reads the learning rate and the Adam step of the update
    # from a device schedule (flat.FusedClipAdam.ensure_window fills it once per 256 updates by stepping the scheduler
    # ahead on a saved state) at a device cursor it advances itself, so a replay is the next update's complete step.
    # Slot graphs are keyed by those pointers.  A slot's first update runs eagerly and warms up workspaces and BLAS
    # handles; the second captures; later ones replay.
    graph_max_rows = 8192
    graph_max_slots = 64   # captured slot graphs per learner; beyond it (e.g. unstable input pointers) stay eager

    def _graph_ok(self, obs):
        # not while ops.TIMER records events: a captured record would be replayed without re-appending its event
        return (getattr(self, "graph_updates", False) and self.grad_sync is None and isinstance(obs, torch.Tensor)
                and obs.is_cuda and obs.shape[0] <= self.graph_max_rows and not getattr(self, "_graph_failed", False)
                and not ops.TIMER.enabled
                and len(self.__dict__.get("_slot_graphs", ())) < self.graph_max_slots)

    def _step_key(self):
        """What a captured update bakes in besides its inputs: the parameter / gradient pointers, the fused optimizer's
        buffers (flat params and grads, Adam moments, schedule table + cursor, norm output) and the K9 constants
        (max_norm, clipping, betas, eps).  Re-homed parameters or a changed hyper-parameter give a new key, so a stale
        graph is never replayed against freed memory or old constants."""
        ptr = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        fused = getattr(self, "fused_opt", None)
        fk = ()
        if fused is not None:
            fk = (ptr(fused.fs.param), ptr(fused.fs.flat), ptr(fused.exp_avg), ptr(fused.exp_avg_sq),
                  ptr(getattr(fused, "_sched", None)), ptr(getattr(fused, "_cursor", None)),
                  ptr(getattr(fused, "total_norm", None)))
        g = self.optimizer.param_groups[0]
        b1, b2 = g.get("betas", (0.9, 0.999))
        return (tuple(p.data_ptr() for p in self._params) + tuple(ptr(p.grad) for p in self._params) + fk
                + (float(self._max_norm) if self._max_norm is not None else None, bool(self._use_clip), float(b1),
                   float(b2), float(g.get("eps", 0.0))))

    def _slot_key(self, obs, idx, act, adv, ret, old_logp, adv_partials):
        ptr = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        # the loss coefficients are kernel arguments baked into a capture: part of the key
        return (ptr(obs), tuple(obs.shape), ptr(idx), -1 if idx is None else idx.shape[0], ptr(act), ptr(adv),
                ptr(ret), ptr(old_logp), ptr(adv_partials), float(self.clip_range), float(self.vf_coef),
                float(self.ent_coef)) + self._step_key()

    def _graphed_mlp_update(self, fm, obs, idx, act, adv, ret, old_logp, adv_partials, pre=None, k9=None):
        """k9: the device part of the clip + Adam step (xpa_clip_adam_step_sched), run after the backward and captured
        with it; the caller does the host bookkeeping."""
        key = self._slot_key(obs, idx, act, adv, ret, old_logp, adv_partials)
        graphs = self.__dict__.setdefault("_slot_graphs", {})
        ent = graphs.get(key)
        if ent is None:                     # first use of this slot: eager (warm-up)
            graphs[key] = "warm"
            if pre is not None:
                pre()
            out = self._mlp_update(fm, obs, idx, act, adv, ret, old_logp, adv_partials, step=False)
            if k9 is not None:
                k9()
            return out
        if ent == "warm":
            if self.__dict__.get("_graph_pool") is None:
                self._graph_pool = torch.cuda.graph_pool_handle()
            g = torch.cuda.CUDAGraph()
            # host-side state a failed capture could leave half-built: restored before the eager retry
            saved = (self._ws, dict(fm._partials), fm._hws)
            try:
                with torch.cuda.graph(g, pool=self._graph_pool):
                    if pre is not None:
                        pre()
                    out = self._mlp_update(fm, obs, idx, act, adv, ret, old_logp, adv_partials, step=False)
                    if k9 is not None:
                        k9()
            except Exception:               # a launch that cannot be captured: stay eager from here on
                self._graph_failed = True
                torch.cuda.synchronize()
                self._ws, fm._partials, fm._hws = saved[0], saved[1], saved[2]
                fm._cq.reset()              # queued finalizes of the aborted capture (capture-pool partials)
                fm._cq_early.reset()
                del graphs[key]
                if pre is not None:
                    pre()
                out = self._mlp_update(fm, obs, idx, act, adv, ret, old_logp, adv_partials, step=False)
                if k9 is not None:
                    k9()
                return out
            graphs[key] = ent = (g, out, self._ws)   # the graph writes into this workspace: keep it alive
        ent[0].replay()
        return ent[1]

    # ---- K30: the whole small-MLP update in one launch (C1) ----------------------------------------------------
    def small_policy_layers(self):
        """((l0, l1, la, l2, lc), code, slope) when the policy is a Categorical actor-critic of one representation
        layer and one hidden layer per head, all with the same activation — the shape K30 (update) and K32 (rollout
        step) take — else None."""
        if self.dist != "categorical":
            return None
        fm = self._fused_mlp()
        if fm is None or len(fm.rep) != 1 or len(fm.actor) != 2 or len(fm.critic) != 2:
            return None
        (l0, c0, s0), (l1, c1, s1), (la, ca, _), (l2, c2, s2), (lc, cc, _) = (fm.rep[0], fm.actor[0], fm.actor[1],
                                                                              fm.critic[0], fm.critic[1])
        if not (c0 == c1 == c2 and s0 == s1 == s2 and ca == 0 and cc == 0 and lc.out_features == 1):
            return None
        return (l0, l1, la, l2, lc), c0, s0

    def small_update_ok(self, obs_flat, batch):
        """True when a minibatch of `batch` rows of obs_flat [n_rows, d] can take K30 (xpa_small_mlp_update): the
        small_policy_layers shape, flat parameters with the fused Adam, no data-parallel gradient sync, and the LDS
        budget."""
        if not getattr(self, "small_updates", True) or self.grad_sync is not None:
            return False
        fused = getattr(self, "fused_opt", None)
        layers = self.small_policy_layers()
        if layers is None or fused is None or fused.fs.numel % 4:
            return False
        if not (isinstance(obs_flat, torch.Tensor) and obs_flat.is_cuda and obs_flat.dim() == 2
                and obs_flat.dtype == torch.float32 and obs_flat.stride(1) == 1):
            return False
        (l0, l1, la, l2, lc), _, _ = layers
        h0, h1, h2, k = l0.out_features, l1.out_features, l2.out_features, la.out_features
        if any(h % 32 or h > 256 for h in (h0, h1, h2)) or not 2 <= k <= 16 or l0.in_features != obs_flat.shape[1] \
                or l0.in_features > 32:
            return False
        rows = 32 if getattr(self, "small_split", True) and 32 < batch <= 512 else batch   # per workgroup
        return int(ops.lib().xpa_small_mlp_lds_floats(rows, l0.in_features, h0, h1, h2, k)) <= 40704

    def _small_launch(self, obs_flat, idx, act, adv, ret, old_logp, use_advnorm, scalars=None):
        """One K30 launch (capturable): reads lr / Adam step at the schedule cursor and advances it.  scalars: the
        8-float destination of the loss scalars (default: the learner's shared one)."""
        fm, fused = self._fused_mlp(), self.fused_opt
        (l0, code, slope), (l1, _, _), (la, _, _), (l2, _, _), (lc, _, _) = (fm.rep[0], fm.actor[0], fm.actor[1],
                                                                             fm.critic[0], fm.critic[1])
        if getattr(self, "_small_scalars", None) is None:
            self._small_scalars = torch.zeros(8, dtype=torch.float32, device=obs_flat.device)
        g = self.optimizer.param_groups[0]
        b1, b2 = g["betas"]
        max_norm = float(self._max_norm) if self._use_clip else -1.0
        a = _lib.XpaSmallMlpArgs()
        a.batch, a.d_in, a.h0, a.h1, a.h2, a.k = (idx.shape[0], l0.in_features, l0.out_features, l1.out_features,
                                                  l2.out_features, la.out_features)
        a.act_code, a.algo, a.use_advnorm, a.n_sched = code, ops.ALGO[self.algo], int(bool(use_advnorm)), \
            fused.SCHED_WINDOW
        a.slope, a.clip_range, a.vf_coef, a.ent_coef = slope, float(self.clip_range), float(self.vf_coef), \
            float(self.ent_coef)
        a.max_norm, a.beta1, a.beta2, a.eps = max_norm, float(b1), float(b2), float(g["eps"])
        a.obs, a.obs_ld, a.idx, a.n_rows = obs_flat.data_ptr(), obs_flat.stride(0), idx.data_ptr(), obs_flat.shape[0]
        a.actions, a.adv, a.ret = act.data_ptr(), adv.data_ptr(), ret.data_ptr()
        a.old_logp = old_logp.data_ptr() if old_logp is not None else None
        a.W0, a.b0, a.W1, a.b1 = l0.weight.data_ptr(), l0.bias.data_ptr(), l1.weight.data_ptr(), l1.bias.data_ptr()
        a.W2, a.b2, a.Wa, a.ba = l2.weight.data_ptr(), l2.bias.data_ptr(), la.weight.data_ptr(), la.bias.data_ptr()
        a.Wc, a.bc = lc.weight.data_ptr(), lc.bias.data_ptr()
        a.gW0, a.gb0, a.gW1, a.gb1 = (l0.weight.grad.data_ptr(), l0.bias.grad.data_ptr(), l1.weight.grad.data_ptr(),
                                      l1.bias.grad.data_ptr())
        a.gW2, a.gb2, a.gWa, a.gba = (l2.weight.grad.data_ptr(), l2.bias.grad.data_ptr(), la.weight.grad.data_ptr(),
                                      la.bias.grad.data_ptr())
        a.gWc, a.gbc = lc.weight.grad.data_ptr(), lc.bias.grad.data_ptr()
        a.param, a.grad = fused.fs.param.data_ptr(), fused.fs.flat.data_ptr()
        a.exp_avg, a.exp_avg_sq, a.n = fused.exp_avg.data_ptr(), fused.exp_avg_sq.data_ptr(), fused.fs.numel
        a.sched, a.cursor = fused._sched.data_ptr(), fused._cursor.data_ptr()
        out = self._small_scalars if scalars is None else scalars
        a.scalars, a.total_norm_out = out.data_ptr(), fused.total_norm.data_ptr()
        st = getattr(self, "small_stamps", None)   # diagnostics: int64 [16] of phase timestamps (tools/k30_stamps.py)
        a.stamps = st.data_ptr() if st is not None else None
        # split form: one workgroup per 32 minibatch rows + a finalize launch (small_split = False: one workgroup)
        B = idx.shape[0]
        G = (B + 31) // 32 if getattr(self, "small_split", True) and 32 < B <= 512 else 1
        a.n_groups = G
        if G > 1:
            ws = self.__dict__.setdefault("_small_split_ws", {})
            if G not in ws:   # zero-filled once: elements no gradient view covers stay 0
                ws[G] = (torch.zeros((G, fused.fs.numel), dtype=torch.float32, device=obs_flat.device),
                         torch.zeros((G, 8), dtype=torch.float64, device=obs_flat.device))
            a.grad_part, a.loss_part = ws[G][0].data_ptr(), ws[G][1].data_ptr()
        _lib.check(ops.lib().xpa_small_mlp_update(ctypes.byref(a), ops._stream(obs_flat.device)),
                   "xpa_small_mlp_update")
        return out

    def small_update(self, obs_flat, idx, act, adv, ret, old_logp=None, use_advnorm=True):
        """One minibatch update through K30 (eager): the device part, then the host bookkeeping of the step."""
        fused = self.fused_opt
        if not fused.sched_enabled:
            fused.enable_sched()
        fused.ensure_window(self.scheduler)
        self.iterations += 1
        out = self._small_launch(obs_flat, idx, act, adv, ret, old_logp, use_advnorm)
        fused.host_step()
        if self.scheduler is not None:
            self.scheduler.step()
        return out

    def small_epoch(self, obs_flat, batches, use_advnorm, keep_all=False):
        """An epoch of K30 updates, batches = [(idx, act, adv, ret, old_logp), ...]: eager the first time a batch
        layout is seen, then captured once as one graph (the launches read the schedule at the device cursor) and
        replayed.  Returns the per-update loss-scalar tensors (see update_epoch for keep_all)."""
        fused = self.fused_opt
        if not fused.sched_enabled:
            fused.enable_sched()
        ptr = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        key = (ptr(obs_flat), tuple(obs_flat.shape), bool(use_advnorm), float(self.clip_range), float(self.vf_coef),
               float(self.ent_coef), bool(getattr(self, "small_split", True))) + \
            tuple((ptr(b[0]), b[0].shape[0], ptr(b[1]), ptr(b[2]), ptr(b[3]), ptr(b[4])) for b in batches) + \
            self._step_key()
        graphs = self.__dict__.setdefault("_small_graphs", {})
        ent = graphs.get(key)
        # bounded like the slot graphs: a caller whose pointers never repeat stays eager instead of growing the cache
        graphed = getattr(self, "graph_updates", False) and not getattr(self, "_graph_failed", False) \
            and len(batches) <= fused.SCHED_WINDOW and (ent is not None or len(graphs) < self.graph_max_slots)
        if ent is None or not graphed:
            outs = []
            for b in batches:
                out = self.small_update(obs_flat, *b, use_advnorm=use_advnorm)
                outs.append(out.clone() if keep_all else out)
            if graphed:
                graphs[key] = "warm"
            return outs
        fused.ensure_window(self.scheduler, need=len(batches))
        if ent == "warm":
            if self.__dict__.get("_graph_pool") is None:
                self._graph_pool = torch.cuda.graph_pool_handle()
            g = torch.cuda.CUDAGraph()
            # every update writes its loss scalars into its own row (no per-update copy inside the graph)
            rows = torch.zeros((len(batches), 8), dtype=torch.float32, device=obs_flat.device)
            try:
                with torch.cuda.graph(g, pool=self._graph_pool):
                    outs = [self._small_launch(obs_flat, *b, use_advnorm=use_advnorm, scalars=rows[i])
                            for i, b in enumerate(batches)]
            except Exception:
                self._graph_failed = True
                torch.cuda.synchronize()
                del graphs[key]
                return self.small_epoch(obs_flat, batches, use_advnorm, keep_all)
            graphs[key] = ent = (g, outs)
        ent[0].replay()
        for _ in batches:
            self.iterations += 1
            fused.host_step()
            if self.scheduler is not None:
                self.scheduler.step()
        return [o.clone() for o in ent[1]] if keep_all else list(ent[1])

    def update_epoch(self, batches, keep_all=False):
        """One epoch of minibatch updates, batches = [(obs, idx, act, adv, ret, old_logp, adv_partials, pre), ...].
        Once every minibatch slot of the epoch has its captured slot graph (K9 inside), the whole sequence is captured
        once more as ONE graph keyed by the slots, and later epochs are one replay (the epoch's host work is then the
        permutation launch before it and the per-update bookkeeping after it).  Otherwise the updates run one by one
        through update_fused.  Returns the per-update loss-scalar tensors (keep_all False: only the last is guaranteed
        to hold its own update's values — the eager updates share their workspace's scalars)."""
        fm = self._fused_mlp()
        fused = getattr(self, "fused_opt", None)
        slots = self.__dict__.get("_slot_graphs", {})
        keys = [self._slot_key(b[0], b[1], b[2], b[3], b[4], b[5], b[6]) for b in batches] \
            if fm is not None and not fm.fused_heads else None
        ready = (keys is not None and fused is not None and fused.sched_enabled and getattr(self, "graph_k9", True)
                 and getattr(self, "graph_epochs", True) and all(self._graph_ok(b[0]) for b in batches)
                 and all(isinstance(slots.get(k), tuple) for k in keys) and len(batches) <= fused.SCHED_WINDOW)
        if not ready:
            return self._eager_epoch(batches, keep_all)
        epochs = self.__dict__.setdefault("_epoch_graphs", {})
        ekey = tuple(keys)
        fused.ensure_window(self.scheduler, need=len(batches))
        ent = epochs.get(ekey)
        if ent is None:
            g = torch.cuda.CUDAGraph()
            # host-side state a failed capture could leave pointing into the aborted capture's pool (a ragged last
            # minibatch reallocates the workspace inside it): restored before the eager fallback
            saved = (self._ws, dict(fm._partials), fm._hws)
            try:
                with torch.cuda.graph(g, pool=self._graph_pool):
                    outs = []
                    for (obs, idx, act, adv, ret, old_logp, adv_partials, pre) in batches:
                        if pre is not None:
                            pre()
                        out = self._mlp_update(fm, obs, idx, act, adv, ret, old_logp, adv_partials, step=False)
                        # every update of the epoch writes the same workspace: each one's scalars copied out in-graph
                        outs.append(out.clone())
                        fused.launch_sched(self._max_norm if self._use_clip else None)
            except Exception:
                # nothing of the aborted capture ran: stay with the slot graphs from here on
                self.graph_epochs = False
                torch.cuda.synchronize()
                self._ws, fm._partials, fm._hws = saved
                fm._cq.reset()
                fm._cq_early.reset()
                return self._eager_epoch(batches, keep_all)
            epochs[ekey] = ent = (g, outs)
        ent[0].replay()
        for _ in batches:
            self.iterations += 1
            fused.host_step()
            if self.scheduler is not None:
                self.scheduler.step()
        # the graph's scalar buffers are rewritten by the next replay: copies when every update's values are kept
        return [o.clone() for o in ent[1]] if keep_all else list(ent[1])

    def _eager_epoch(self, batches, keep_all):
        outs = []
        for b in batches:
            out = self.update_fused(*b[:7], pre=b[7])
            outs.append(out.clone() if keep_all else out)
        return outs

    def _mlp_update(self, fm, obs, idx, act, adv, ret, old_logp, adv_partials, step):
        """Explicit forward (fused_mlp) + K2 loss + explicit backward into the flat gradient (+ K9 when step)."""
        head, logstd, v, ctx = fm.forward(obs)
        if self._ws is None or self._ws.batch != head.shape[0]:
            self._ws = ops.LossWorkspace(head.shape[0], head.shape[1], head.device, self.dist)
        scalars, dh, _, dv = ops.policy_loss(self.algo, self.dist, head, logstd, v, act, adv, ret,
                                             old_logp=old_logp, idx=idx, adv_partials=adv_partials,
                                             clip_range=self.clip_range, vf_coef=self.vf_coef,
                                             ent_coef=self.ent_coef, ws=self._ws,
                                             d_logstd_out=logstd.grad if logstd is not None else None)
        fm.backward(ctx, dh, dv)       # writes every parameter gradient into the flat buffer
        if step:
            self._sync_clip_step()
        return scalars

    def enable_fast_path(self, fused_optimizer=True):
        """Flat parameters/gradients and the fused clip+Adam kernel (xuanpolicy_amd.flat)."""
        from .distributed import attach_flat_grads
        if getattr(self, "flat_grads", None) is None:
            attach_flat_grads(self, allreduce=True, fused_optimizer=fused_optimizer)
        return self

    def _info(self, scalars):
        s = scalars.detach().cpu().tolist()
        info = {"actor-loss": s[0], "critic-loss": s[1], "entropy": s[2],
                "learning_rate": self.optimizer.param_groups[0]["lr"], "predict_value": s[5]}
        if self.algo == "ppo":
            info["clip_ratio"] = s[4]
        return info

    @staticmethod
    def _t(x, device, dtype=torch.float32):
        if isinstance(x, torch.Tensor):
            return x.to(device=device, dtype=dtype).contiguous()
        import numpy as np
        return torch.as_tensor(np.asarray(x), dtype=dtype, device=device).contiguous()

    @classmethod
    def _obs(cls, x, device):
        """Observations: raw uint8 frames stay uint8 (the CNN path converts them on device, K20), the rest float32."""
        import numpy as np
        if (isinstance(x, torch.Tensor) and x.dtype == torch.uint8) or (isinstance(x, np.ndarray) and x.dtype == np.uint8):
            return cls._t(x, device, torch.uint8)
        return cls._t(x, device)

    def _device(self):
        return next(self.policy.parameters()).device

    def _check_actions(self, act_batch):
        """Categorical.log_prob validates its argument and raises on an action outside [0, n) (the loss kernel
        clamps instead, loss.hip): host-supplied batches are checked here, before the upload.  Device tensors come
        from the device rollout, which only writes in-range actions, and are not synced for the check."""
        if self.dist != "categorical" or (isinstance(act_batch, torch.Tensor) and act_batch.is_cuda):
            return
        import numpy as np
        a = act_batch.numpy() if isinstance(act_batch, torch.Tensor) else np.asarray(act_batch)
        n = int(getattr(self.policy, "action_dim", 0) or 0)
        if a.size and (not np.all(np.isfinite(a)) or a.min() < 0 or (n and a.max() >= n) or np.any(a != np.floor(a))):
            raise ValueError(f"categorical actions must be integers in [0, {n}); got range [{a.min()}, {a.max()}]")


class PPOCLIP_Learner(_FusedPolicyGradient):
    """ppoclip_learner.py:4-65."""
    algo = "ppo"

    def __init__(self, policy, optimizer, scheduler=None, device=None, model_dir="./", vf_coef=0.25, ent_coef=0.005,
                 clip_range=0.25, clip_grad_norm=0.25, use_grad_clip=True):
        super().__init__(policy, optimizer, scheduler, device, model_dir, vf_coef, ent_coef, clip_range,
                         clip_grad_norm, use_grad_clip)
        self.clip_grad_norm, self.use_grad_clip = clip_grad_norm, use_grad_clip

    def update(self, obs_batch, act_batch, ret_batch, value_batch, adv_batch, old_logp):
        dev = self._device()
        self._check_actions(act_batch)
        scalars = self.update_fused(self._obs(obs_batch, dev), None, self._t(act_batch, dev).reshape(-1),
                                    self._t(adv_batch, dev), self._t(ret_batch, dev), self._t(old_logp, dev))
        return self._info(scalars)


class A2C_Learner(_FusedPolicyGradient):
    """a2c_learner.py:4-50 (always clips the gradient norm, a2c_learner.py:34)."""
    algo = "a2c"

    def __init__(self, policy, optimizer, scheduler=None, device=None, model_dir="./", vf_coef=0.25, ent_coef=0.005,
                 clip_grad=None):
        if clip_grad is None:   # the reference's clip_grad_norm_(..., None) fails at its first update
            raise ValueError("A2C_Learner needs clip_grad (a2c_learner.py:34 always clips)")
        super().__init__(policy, optimizer, scheduler, device, model_dir, vf_coef, ent_coef, 0.0, clip_grad, True)
        self.clip_grad = clip_grad

    def update(self, obs_batch, act_batch, ret_batch, adv_batch):
        dev = self._device()
        self._check_actions(act_batch)
        scalars = self.update_fused(self._obs(obs_batch, dev), None, self._t(act_batch, dev).reshape(-1),
                                    self._t(adv_batch, dev), self._t(ret_batch, dev))
        return self._info(scalars)


REGISTRY = {"PPO_Clip": PPOCLIP_Learner, "A2C": A2C_Learner}


class PerDQN_Learner(Learner):
    """perdqn_learner.py:4-48 (same constructor, update(obs, act, rew, next, terminal) -> (|TD|, info)).

    The Q-network forwards (eval on obs, target on next) and the backward stay in PyTorch-ROCm (MIOpen
    convolutions, hipBLASLt GEMMs); the tensor algebra between them — TD target with max over the target Q row,
    the gathered prediction, MSE, its gradient w.r.t. evalQ and the |TD| priorities — is K19 (xpa_dqn_td_loss,
    one launch).  |TD| stays on the device (a float32 tensor the device PerOffPolicyBuffer.update_priorities
    takes as it is); the reference returns a NumPy array.  Hard target copy every sync_frequency updates."""

    def __init__(self, policy, optimizer, scheduler=None, device=None, model_dir="./", gamma=0.99,
                 sync_frequency=100):
        self.gamma = gamma
        self.sync_frequency = sync_frequency
        super().__init__(policy, optimizer, scheduler, device, model_dir)
        self._err = None

    def _f32(self, x, dev):
        if isinstance(x, torch.Tensor):
            return x.to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
        return torch.as_tensor(x, dtype=torch.float32, device=dev).reshape(-1).contiguous()

    def _fused_q(self):
        """Explicit Q-network forward / backward (fused_cnn.FusedQNetwork) for CNN Q-networks on uint8 frames."""
        fq = getattr(self, "_fq", None)
        if fq is None:
            fq = False
            dev = next(self.policy.parameters()).device
            if getattr(self, "fused_cnn_enabled", True) and dev.type == "cuda" and hasattr(self.policy, "eval_Qhead"):
                from .fused_cnn import FusedQNetwork
                try:
                    fq = FusedQNetwork(self.policy)
                except ValueError:
                    fq = False
            self._fq = fq
        return fq or None

    def q_values(self, obs):
        """evalQ of the eval network (the agent's action selection)."""
        fq = self._fused_q()
        if fq is not None and isinstance(obs, torch.Tensor) and obs.dtype == torch.uint8 and obs.is_cuda:
            return fq.forward(obs.contiguous())[0]
        with torch.no_grad():
            return self.policy(obs)[2]

    def update(self, obs_batch, act_batch, rew_batch, next_batch, terminal_batch, sync_info=True):
        self.iterations += 1
        fq = self._fused_q()
        fused = (fq is not None and isinstance(obs_batch, torch.Tensor) and obs_batch.dtype == torch.uint8
                 and obs_batch.is_cuda and isinstance(next_batch, torch.Tensor) and next_batch.dtype == torch.uint8)
        if fused:   # K20 frames, MIOpen convs + K21, K23 max pool, Q head GEMMs; backward K24 / K22 + MIOpen
            evalQ, ctx = fq.forward(obs_batch.contiguous())
            targetQ = fq.target(next_batch.contiguous())
        else:
            _, _, evalQ = self.policy(obs_batch)
            with torch.no_grad():
                _, _, targetQ = self.policy.target(next_batch)
        dev = evalQ.device
        if self._err is None:
            self._err = torch.zeros(1, dtype=torch.int32, device=dev)
        dQ, td_abs, sc = ops.dqn_td_loss(evalQ.detach(), targetQ, self._f32(act_batch, dev), self._f32(rew_batch, dev),
                                         self._f32(terminal_batch, dev), self.gamma, err=self._err)
        if fused:
            fq.backward(ctx, dQ)           # overwrites every eval-network gradient
        else:
            self.optimizer.zero_grad()
            evalQ.backward(dQ)
        self.optimizer.step()
        if self.scheduler is not None:
            self.scheduler.step()
        if self.iterations % self.sync_frequency == 0:
            self.policy.copy_target()
        lr = self.optimizer.param_groups[0]["lr"]
        if not sync_info:   # the agent's hot loop: scalars stay on the device
            return td_abs, {"Qloss": sc[0], "learning_rate": lr, "predictQ": sc[1]}
        q = sc.cpu().tolist()
        return td_abs, {"Qloss": q[0], "learning_rate": lr, "predictQ": q[1]}

REGISTRY["PerDQN"] = PerDQN_Learner
