"""Explicit forward/backward of the actor-critic MLP for the learner's hot path (no autograd graph).

Reference network: representation Basic_MLP -> ActorNet (mu or logits) and CriticNet, each a chain of
mlp_block = Linear -> activation (xuance/torch/representations/mlp.py:21-51,
xuance/torch/policies/gaussian.py:8-51, categorical.py:16-58, xuance/torch/utils/layers.py:8-24).
PPOCLIP_Learner.update runs loss.backward() through it (ppoclip_learner.py:46).  Two explicit paths
write every parameter gradient into the flat gradient buffer (flat.FlatState):
  * forward_hidden() + loss_backward() (the learner's fast path): K13 for the first layer, ONE GEMM
    for the actor|critic hidden layers when FlatState placed them back to back (head_placement), K12
    for both heads (activation, output layer, loss, head backward), then one dW and one dX GEMM;
  * forward() + backward(d_head, d_v) after the K2 loss kernel, for other shapes, with:
  * hipBLASLt GEMMs for dX (the trunk's two heads accumulate with one addmm: no separate add pass);
  * split-K batched GEMMs for dW = dZ^T X written with sum(out=grad view) (see policies._splitk_splits);
  * K10 xpa_act_bwd_colsum: activation backward + bias-gradient column sums in one pass over [B, H]
    (output layers: column sums only), xpa_colsum_finalize into the bias-gradient views.
Forward: F.linear (GEMM + bias epilogue) then the activation in place; the activation OUTPUTS are
kept (LeakyReLU/ReLU/tanh derivatives are functions of the output), no pre-activation copies.
Every parameter gradient is overwritten each update, so no zeroing pass is needed.
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib, ops
from .policies import Basic_Identical, _splitk_splits, policy_discrete


def _act_code(m):
    if m is None:
        return 0, 0.0
    if isinstance(m, nn.LeakyReLU):
        return 1, float(m.negative_slope)
    if isinstance(m, nn.ReLU):
        return 1, 0.0
    if isinstance(m, nn.Tanh):
        return 2, 0.0
    raise ValueError("unsupported activation %r" % type(m).__name__)


def _parse(seq):
    mods = list(seq)
    layers, i = [], 0
    while i < len(mods):
        lin = mods[i]
        if not isinstance(lin, nn.Linear) or lin.bias is None:
            raise ValueError("expected Linear with bias, got %r" % type(lin).__name__)
        act = None
        if i + 1 < len(mods) and not isinstance(mods[i + 1], nn.Linear):
            act = mods[i + 1]
            i += 2
        else:
            i += 1
        layers.append((lin,) + _act_code(act))
    return layers


def _rep_layers(rep):
    """The representation's Linear(+activation) chain, recognised by structure rather than class, so the reference's
    own Basic_MLP / Basic_Identical (xuance/torch/representations/mlp.py:5-51: a `.model` nn.Sequential of mlp_block
    Linear + activation pairs, empty for the identity) take the same path as ours; anything else (convolutions,
    normalisation layers) raises ValueError and the learner keeps the generic path."""
    model = getattr(rep, "model", None)
    if isinstance(model, nn.Sequential):
        return _parse(model)
    if isinstance(rep, Basic_Identical):
        return []
    raise ValueError("representation %r has no explicit backward" % type(rep).__name__)


def _head_layers(policy):
    discrete = policy_discrete(policy)
    actor = [m for m in (policy.actor.model if discrete else policy.actor.mu) if isinstance(m, nn.Linear)]
    critic = [m for m in policy.critic.model if isinstance(m, nn.Linear)]
    return actor, critic


def head_placement(policy):
    """FlatState placement groups that let the actor's and the critic's hidden layer run as one
    [512, in] layer: both heads must be [Linear(in, 256) + act] -> Linear(256, K) on the same input."""
    try:
        actor, critic = _head_layers(policy)
    except AttributeError:
        return []
    if (len(actor) != 2 or len(critic) != 2 or actor[0].in_features != critic[0].in_features
            or actor[0].out_features != ops.HEAD_HIDDEN or critic[0].out_features != ops.HEAD_HIDDEN
            or actor[0].bias is None or critic[0].bias is None):
        return []
    return [[actor[0].weight, critic[0].weight], [actor[0].bias, critic[0].bias]]


class Rows:
    """The minibatch rows `idx` of a flat [n_rows, d] buffer, handed to the fused path instead of a gathered copy:
    K13's gather forms (xpa_thin_linear_act_fwd_gather / _bwd_gather) read them through the permutation."""

    def __init__(self, flat, idx):
        self.flat, self.idx = flat, idx
        self.gathered = None   # set by the gather forward: the rows as a contiguous [B, d] copy
        self.trunk = None      # K16X: (gathered rows, W0, b0, slope, h out) when the head launches form h
        self.hsign = None      # K13's sign bits of h (int32 [B, 8]) for K42S
        self.wide_direct = False   # r05: the wide trunk read these rows through idx (no gathered copy)
        self.shape = (idx.shape[0], flat.shape[1])
        self.device = flat.device
        self.dtype = flat.dtype


def _vec4_rows(t):
    """The split GEMMs (K40 / K41 / K42) read operands as 16-B vectors: unit column stride, a row stride that is a
    multiple of 4 floats and a 16-B aligned base.  Anything else takes the f32 library / chain path."""
    return t.stride(1) == 1 and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0


class FusedActorCritic:
    """Built from a Gaussian/Categorical actor-critic policy whose parameters live in a FlatState
    (pass it as `flat` to use the paired actor|critic hidden layer when head_placement applied)."""

    def __init__(self, policy, flat=None):
        self.rep = _rep_layers(policy.representation)
        self.discrete = policy_discrete(policy)
        self.actor = _parse(policy.actor.model if self.discrete else policy.actor.mu)
        self.critic = _parse(policy.critic.model)
        self.logstd = None if self.discrete else policy.actor.logstd
        self.use_head_kernel = True
        # K12 (fused head + loss + backward) when both heads end in [Linear(., 256) + act] -> Linear(256, K)
        k = self.actor[-1][0].out_features
        self.fused_heads = (self._head_fusable(self.actor) and self._head_fusable(self.critic)
                            and k <= ops.HEAD_KMAX and (k >= 2 or not self.discrete))
        self._hws = None
        # K13 for the first representation layer when its input is narrow (observation width <= 64)
        self.thin0 = (len(self.rep) > 0 and self.rep[0][0].in_features <= 64
                      and self.rep[0][0].out_features == ops.HEAD_HIDDEN)
        # r05 (C4): one WIDE representation layer (d_in > 64, d_in % 4 == 0, identity / LeakyReLU) on the split GEMMs —
        # K40F forward from the zero-padded gathered rows (+ h's sign bits), K42W / K42C-dz backward to dz1, K41V dW^T
        # slices finalized transposed into W0's gradient (_wide_on)
        self.wide0 = (len(self.rep) == 1 and not self.thin0 and self.rep[0][0].out_features == ops.HEAD_HIDDEN
                      and self.rep[0][0].in_features % 4 == 0 and self.rep[0][0].in_features <= 4096
                      and self.rep[0][1] in (0, 1))
        self.pair = None
        if self.fused_heads and flat is not None and len(self.actor) == 2 and len(self.critic) == 2:
            la, lc = self.actor[0][0], self.critic[0][0]
            if la.in_features == lc.in_features:
                w = flat.span([la.weight, lc.weight])
                b = flat.span([la.bias, lc.bias])
                if w is not None and b is not None:
                    n_in = la.in_features
                    self.pair = (w[0].view(2 * ops.HEAD_HIDDEN, n_in), b[0], w[1].view(2 * ops.HEAD_HIDDEN, n_in), b[1])
        # K16: the paired hidden layers' forward GEMM inside the head kernels (fp32 MFMA), when their
        # input is 256 wide; z is then never materialised.
        self.gemm_heads = self.pair is not None and self.actor[0][0].in_features == ops.HEAD_HIDDEN
        # K16X: the trunk (one thin layer, d_in <= 20, the heads' activation) inside the K16 launches as well, so the
        # update's trunk output h is formed in LDS and written once (by the actor launch) instead of K13's write + two
        # K16 reads; minibatch rows from Rows only (the gather-only K13 form supplies the rows and the adv moments)
        self.trunk_heads = (self.gemm_heads and self.thin0 and len(self.rep) == 1
                            and self.rep[0][0].in_features <= ops.TRUNK_DMAX and k <= 8
                            and self.rep[0][1:] == self.actor[-2][1:] == self.critic[-2][1:])
        # measured slower at C2 (r03): off unless asked for (bench.py --trunk-heads on)
        self.use_trunk_heads = False
        n_params = sum(1 for _ in policy.parameters())
        n_cov = 2 * (len(self.rep) + len(self.actor) + len(self.critic)) + (0 if self.discrete else 1)
        if n_params != n_cov:
            raise ValueError("policy has parameters outside the Linear chains")
        self._partials = {}
        self._cq = ops.ColsumQueue()
        self._cq_early = ops.ColsumQueue()
        self.early_grad_sync = None   # data-parallel: callable(grad_view) starting an early all-reduce
        self._sq = None
        self.sq_ready = None
        self._params = list(policy.parameters())
        self._n_params = None

    @staticmethod
    def _head_fusable(layers):
        return (len(layers) >= 2 and layers[-1][1] == 0 and layers[-2][0].out_features == ops.HEAD_HIDDEN
                and layers[-1][0].in_features == ops.HEAD_HIDDEN)

    # ------------------------------------------------------------------------------------------------
    @staticmethod
    def _chain_forward(layers, x):
        outs = []
        h = x
        for lin, code, slope in layers:
            h = F.linear(h, lin.weight, lin.bias)
            if code == 1:
                F.leaky_relu(h, slope, inplace=True)
            elif code == 2:
                h.tanh_()
            outs.append(h)
        return outs

    def rows_ok(self, flat):
        """True when the update can take Rows(flat, idx) (K13 with the gather folded in, or the wide trunk's pitched
        gather)."""
        return (self.fused_heads and (self.thin0 or self._wide_on()) and flat.dim() == 2
                and flat.dtype == torch.float32 and flat.stride(1) == 1 and flat.is_cuda
                and (self.thin0 or flat.is_contiguous()))

    WIDE_TRUNK = True   # r05: the wide trunk layer on K40F / K42W / K41V where it applies (bench.py --wide-trunk off: A/B)

    def _wide_on(self):
        return (self.WIDE_TRUNK and self.wide0 and self.fused_heads and ops.S3_GEMMS and self.pair is not None
                and self._dx_split_ok(self.pair[0]))

    WIDE_DIRECT = True   # r05: K40F / K41V read the minibatch rows through idx from the rollout buffer (no gather)

    @staticmethod
    def _wide_mpad(d):
        return (d + 127) // 128 * 128   # K41V's row tiles over the layer's inputs

    WIDE_VIDX_MAX = 1536   # K41V-IDX's LDS index stage (csrc/sgemm3.hip kVIdxMax): rows per slice, rounded to 32

    @classmethod
    def _wide_slices(cls, kp):
        return max(1, 256 // (kp // 128))

    def _wide_direct_ok(self, x, d):
        """The row-index forms apply: the flat buffer's rows are the layer width and readable, finite (zeroed) slack
        follows its last row for the padded columns (buffer.OBS_SLACK), and K41V-IDX's per-slice row count fits its LDS
        index stage (else the pitched gather, which has no such limit).  K40F reads columns d .. kp - 1 of a row from
        the next row and zeroes them before the split (r06), so a non-finite next row does not reach this row's outputs
        (tests/test_gpu_wide_trunk.py::test_row_index_form_ignores_the_next_rows_values)."""
        f = x.flat
        mp = self._wide_mpad(d)
        need = max((d + 15) // 16 * 16, mp) - d
        S = self._wide_slices(mp)
        per = (x.idx.shape[0] + S - 1) // S
        per = (per + 31) // 32 * 32
        return (self.WIDE_DIRECT and f.dim() == 2 and f.is_contiguous() and f.shape[1] == d and d % 4 == 0
                and f.data_ptr() % 16 == 0 and per <= self.WIDE_VIDX_MAX
                and f.untyped_storage().nbytes() // 4 >= f.storage_offset() + f.numel() + need)

    def _wide_forward(self, x, adv, adv_partials):
        """The wide trunk layer's forward on the minibatch rows x = Rows(flat, idx): W0^T's split (zero rows to d_pad),
        then K40F (bias, activation and h's sign bits in the epilogue) reading the rows through idx straight from the
        rollout buffer (+ the advantage moments from a row-less K4); or, where the buffer has no slack, the pitched
        gather into a zero-padded [B, d_pad] buffer first."""
        lin, code, slope = self.rep[0]
        B, d = x.idx.shape[0], lin.in_features
        kp = (d + 15) // 16 * 16
        if self._wide_direct_ok(x, d):
            if adv_partials is not None:   # K4's advantage moments alone (zero-width rows)
                ops.gather_minibatch(x.idx, x.flat[:, :0], adv=adv, adv_partials=adv_partials,
                                     obs_out=x.flat.new_empty((B, 0)))
            x.gathered = None
            x.wide_direct = True
            x.hsign = self._sign_buf(B, x.device)
            wsplit = self._split_buf(kp, "w0t", x.device)
            ops.s3_split_padded(lin.weight.t(), kp, out=wsplit)
            h = torch.empty((B, lin.out_features), dtype=torch.float32, device=x.device)
            ops.s3_gemm_bias_act(x.flat, wsplit, kp, lin.bias, code, slope, out=h, sign=x.hsign, ridx=x.idx)
            return [h]
        key = ("wide_x", B, kp)
        xp = self._partials.get(key)
        if xp is None:   # graph-capture safe: allocated (and its pad zeroed) on first (eager) use
            xp = torch.zeros((B, kp), dtype=torch.float32, device=x.device)
            self._partials[key] = xp
        ops.gather_minibatch_pitched(x.idx, x.flat, xp, adv=adv if adv_partials is not None else None,
                                     adv_partials=adv_partials)
        x.gathered = xp
        x.hsign = self._sign_buf(B, x.device)
        wsplit = self._split_buf(kp, "w0t", x.device)
        ops.s3_split_padded(lin.weight.t(), kp, out=wsplit)
        h = torch.empty((B, lin.out_features), dtype=torch.float32, device=x.device)
        ops.s3_gemm_bias_act(xp, wsplit, kp, lin.bias, code, slope, out=h, sign=x.hsign)
        return [h]

    def _wide_bwd(self, dz, x, crit):
        """K42W (or K42C's dz form with the factored critic): dz1 = (dz . Wh_pair) act'(h) and db0's partials; K41V's
        slices of x_pad^T dz1, finalized transposed (and trimmed to d_in) into W0's gradient."""
        lin, code, slope = self.rep[0]
        B, d = dz.shape[0], lin.in_features
        direct = getattr(x, "wide_direct", False)
        xp = x.gathered
        kp = self._wide_mpad(d) if direct else xp.shape[1]
        S = self._wide_slices(kp)
        key = ("wide_bwd", B, kp, S)
        ws = self._partials.get(key)
        if ws is None:
            G = int(ops.lib().xpa_s3_gemm_trunk_bwd_num_partials(B))
            ws = (torch.empty((B, 256), device=dz.device), torch.empty((G, 256), device=dz.device),
                  torch.empty((S, kp, 256), device=dz.device))
            self._partials[key] = ws
        dz1, pdb, pdw = ws
        k = self.pair[0].shape[0]
        if crit is not None:
            H = ops.HEAD_HIDDEN
            ops.s3_gemm_trunk_bwd_dz(dz, self._split_buf(k, "dx_crit", dz.device), k, x.hsign, code, slope, dz1, pdb,
                                     crit=(H, k - H, crit[0], crit[1], crit[2]))
        else:
            ops.s3_gemm_trunk_bwd_dz(dz, self._split_buf(k, "dx", dz.device), k, x.hsign, code, slope, dz1, pdb)
        if direct:   # K41V through idx from the rollout buffer (rows d .. kp - 1 of the slices: garbage, dropped)
            ops.s3_wgrad(x.flat, dz1, out=pdw, slices=S, aidx=x.idx, m=kp)
        else:
            ops.s3_wgrad(xp, dz1, out=pdw, slices=S)
        self._cq.add(pdw.view(S, -1), lin.weight.grad, tmap=(256, d, d))
        self._cq.add(pdb, lin.bias.grad)
        return True

    def _rep_forward(self, x, norm=None, adv=None, adv_partials=None, defer_trunk=False):
        if isinstance(x, Rows) and not self.thin0:
            if not self._wide_on():
                raise ValueError("Rows input needs the thin (K13) or the wide (K40F) trunk layer")
            return self._wide_forward(x, adv, adv_partials)
        if isinstance(x, Rows):
            # K4's gather folded into K13's x staging (+ the advantage moments when adv_partials is given)
            lin, code, slope = self.rep[0]
            B = x.idx.shape[0]
            h = torch.empty((B, lin.out_features), dtype=torch.float32, device=x.device)
            # the gathered rows are written beside h (4 B x d_in per row) so the backward reads them contiguously
            # (reading them through idx again cost K13's backward 3.3 us per update)
            x.gathered = torch.empty((B, lin.in_features), dtype=torch.float32, device=x.device)
            # K16X: gather-only (h = NULL); the actor head launch forms h and writes it here
            # (only for forward_hidden -> loss_backward, where the K16X launches consume x.trunk; h is unwritten until then)
            deferred = defer_trunk and self.trunk_heads and (self.use_trunk_heads or self._s3r_on()) and len(self.rep) == 1
            if deferred:
                x.trunk = (x.gathered, lin.weight, lin.bias, slope, h)
                if self._s3r_on() and code in (0, 1):   # K16R's sign bits of h for K42S (act' without reading h)
                    x.trunk = x.trunk + (self._sign_buf(B, x.device),)
            x.hsign = None
            if not deferred and defer_trunk and self._sign_on(code):
                # K13 writes h's sign bits beside h: K42S's act' (32 B per row read instead of h's 1 KiB)
                x.hsign = self._sign_buf(B, x.device)
                _lib.check(ops.lib().xpa_thin_linear_act_fwd_gather_sign(
                    code, ops._p(x.flat), x.flat.stride(0), x.flat.shape[0], ops._p(x.idx), B, lin.in_features,
                    lin.out_features, ops._p(lin.weight), ops._p(lin.bias), slope, ops._p(h), h.stride(0),
                    ops._p(adv) if adv_partials is not None else None,
                    ops._p(adv_partials) if adv_partials is not None else None, ops._p(x.gathered),
                    ops._p(x.hsign), ops._stream(x.device)), "xpa_thin_linear_act_fwd_gather_sign")
                return [h] + self._chain_forward(self.rep[1:], h)
            _lib.check(ops.lib().xpa_thin_linear_act_fwd_gather(
                code, ops._p(x.flat), x.flat.stride(0), x.flat.shape[0], ops._p(x.idx), B, lin.in_features,
                lin.out_features, ops._p(lin.weight), ops._p(lin.bias), slope, None if deferred else ops._p(h),
                h.stride(0),
                ops._p(adv) if adv_partials is not None else None,
                ops._p(adv_partials) if adv_partials is not None else None, ops._p(x.gathered),
                ops._stream(x.device)), "xpa_thin_linear_act_fwd_gather")
            return [h] + self._chain_forward(self.rep[1:], h)
        if norm is not None:
            # x RAW: observation normalisation fused into the first layer (xpa_thin_linear_act_fwd_norm);
            # norm = (mean, var, clip, xn_out, col, col_ld, cursor)
            if not self.thin0:
                raise ValueError("fused normalisation needs the thin first layer (K13)")
            lin, code, slope = self.rep[0]
            mean, var, clip, xn, col, col_ld, cursor = norm
            h = torch.empty((x.shape[0], lin.out_features), dtype=torch.float32, device=x.device)
            _lib.check(ops.lib().xpa_thin_linear_act_fwd_norm(
                code, ops._p(x), x.stride(0), x.shape[0], lin.in_features, lin.out_features, ops._p(lin.weight),
                ops._p(lin.bias), slope, ops._p(h), h.stride(0), ops._p(mean), ops._p(var), float(clip), ops._p(xn),
                xn.stride(0), ops._p(col), int(col_ld), ops._p(cursor), ops._stream(x.device)),
                "xpa_thin_linear_act_fwd_norm")
            return [h] + self._chain_forward(self.rep[1:], h)
        if self.thin0 and x.dim() == 2 and x.dtype == torch.float32 and x.stride(1) == 1:
            lin, code, slope = self.rep[0]
            h = torch.empty((x.shape[0], lin.out_features), dtype=torch.float32, device=x.device)
            _lib.check(ops.lib().xpa_thin_linear_act_fwd(code, ops._p(x), x.stride(0), x.shape[0], lin.in_features,
                                                         lin.out_features, ops._p(lin.weight), ops._p(lin.bias), slope,
                                                         ops._p(h), h.stride(0), ops._stream(x.device)),
                       "xpa_thin_linear_act_fwd")
            return [h] + self._chain_forward(self.rep[1:], h)
        return self._chain_forward(self.rep, x)

    def _thin_backward(self, layer, g, h, x):
        lin, code, slope = layer
        rows, din = x.shape[0], lin.in_features
        L = ops.lib()
        key = ("thin", rows, din)
        ws = self._partials.get(key)
        if ws is None:
            G = int(L.xpa_thin_bwd_num_partials(rows))
            ws = (torch.empty((G, lin.out_features * din), device=g.device),
                  torch.empty((G, lin.out_features), device=g.device))
            self._partials[key] = ws
        pdw, pdb = ws
        s = ops._stream(g.device)
        if isinstance(x, Rows) and getattr(x, "gathered", None) is not None:
            x = x.gathered
        if isinstance(x, Rows):
            _lib.check(L.xpa_thin_linear_act_bwd_gather(code, ops._p(g), g.stride(0), ops._p(h), h.stride(0), rows,
                                                        ops._p(x.flat), x.flat.stride(0), x.flat.shape[0],
                                                        ops._p(x.idx), din, lin.out_features, slope, ops._p(pdw),
                                                        ops._p(pdb), s), "xpa_thin_linear_act_bwd_gather")
        else:
            _lib.check(L.xpa_thin_linear_act_bwd(code, ops._p(g), g.stride(0), ops._p(h), h.stride(0), rows,
                                                 ops._p(x), x.stride(0), din, lin.out_features, slope, ops._p(pdw),
                                                 ops._p(pdb), s), "xpa_thin_linear_act_bwd")
        self._cq.add(pdw, lin.weight.grad)
        self._cq.add(pdb, lin.bias.grad)

    @torch.no_grad()
    def forward(self, x):
        rep_outs = self._rep_forward(x)
        s = rep_outs[-1] if rep_outs else x
        a_outs = self._chain_forward(self.actor, s)
        c_outs = self._chain_forward(self.critic, s)
        v = c_outs[-1][:, 0]
        return a_outs[-1], self.logstd, v, (x, rep_outs, s, a_outs, c_outs)

    # ---- rollout-side forwards (K14) ---------------------------------------------------------------
    @property
    def rollout_ok(self):
        return self.pair is not None

    # r05 (K40R): the rollout's paired hidden GEMM on the split; the planes of [Wh_actor^T | Wh_critic^T] are re-split at
    # the start of every rollout (rollout_refresh, outside any captured graph: the weights change only in the update)
    ROLLOUT_SPLIT = True

    def rollout_refresh(self):
        """Split the paired hidden layer's weights for K40R (one launch, before a rollout's first step); afterwards
        rollout_act uses the planes until the next refresh.  A no-op (planes dropped) where K40R does not apply."""
        lin_a, lin_c = self.actor[0][0], self.critic[0][0]
        ok = (self.ROLLOUT_SPLIT and ops.S3_GEMMS and self.pair is not None and self.gemm_heads
              and lin_a.in_features == 256 and lin_a.out_features == 256 and lin_c.out_features == 256)
        if not ok:
            self._roll_split = None
            return
        bufs = self._split_many([(lin_a.weight.t(), "roll_a"), (lin_c.weight.t(), "roll_c")])
        self._roll_split = (bufs[0], bufs[1])

    def _rollout_pair(self, s):
        rs = getattr(self, "_roll_split", None)
        if rs is not None and s.dim() == 2 and s.shape[1] == 256 and _vec4_rows(s):
            return ops.s3_gemm_rows_pair(s, rs[0], rs[1], self.pair[1])
        return F.linear(s, self.pair[0], self.pair[1])

    # r06 (K40T, opt-in: XPA_ROLLOUT_TRUNK=1): with the normalisation fused (norm given), a one-layer thin trunk
    # (d_in <= 18) and K40R's planes, the trunk runs inside the paired hidden GEMM's launch (h never stored).  Measured
    # no faster than K13-norm + K40R (20.4-22.4 vs 20.7 us per env step at C2), so off
    ROLLOUT_TRUNK = os.environ.get("XPA_ROLLOUT_TRUNK", "0") == "1"

    def _rollout_trunk_pair(self, x, norm):
        rs = getattr(self, "_roll_split", None)
        if (not self.ROLLOUT_TRUNK or norm is None or rs is None or not self.thin0 or len(self.rep) != 1
                or x.dim() != 2 or x.dtype != torch.float32 or x.stride(1) != 1):
            return None
        lin, code, slope = self.rep[0]
        if lin.in_features > 18 or lin.out_features != 256:
            return None
        mean, var, clip, xn, col, col_ld, cursor = norm
        return ops.s3_gemm_rows_pair_trunk(x, lin.weight, lin.bias, code, slope, mean, var, clip, xn, col, col_ld,
                                           cursor, rs[0], rs[1], self.pair[1])

    @torch.no_grad()
    def rollout_act(self, x, dist, cursor, seed, buf_act, buf_logp, buf_val, env_in, act_clip=1.0, norm=None,
                    env=None, post=None):
        """Policy step of the rollout: trunk, paired hidden GEMM, then K14 (heads + sample + store).
        norm: see _rep_forward (x is then the raw observation).  env: a device SynthBox env whose step runs
        inside the same K14 launch (ops.rollout_policy_head_synthbox; the caller skips env.step_device()).
        post (with env, r06): K8's post step in that launch too (K14F; ops.rollout_policy_head_synthbox(post=))."""
        z = self._rollout_trunk_pair(x, norm)
        if z is None:
            rep_outs = self._rep_forward(x, norm=norm)
            s = rep_outs[-1] if rep_outs else x
            z = self._rollout_pair(s)
        H = ops.HEAD_HIDDEN
        lin_ao = self.actor[-1][0]
        lin_co = self.critic[-1][0]
        _, code, slope = self.actor[-2]
        if self.critic[-2][1:] != (code, slope):
            raise ValueError("actor and critic hidden activations differ")
        if env is not None:
            ops.rollout_policy_head_synthbox(z[:, :H], z[:, H:], (code, slope), lin_ao.weight, lin_ao.bias,
                                             lin_co.weight, lin_co.bias, self.logstd, cursor, seed, buf_act, buf_logp,
                                             buf_val, env, act_clip, post=post)
            return
        ops.rollout_policy_head(dist, z[:, :H], z[:, H:], (code, slope), lin_ao.weight, lin_ao.bias, lin_co.weight,
                                lin_co.bias, self.logstd, cursor, seed, buf_act, buf_logp, buf_val, env_in, act_clip)

    @torch.no_grad()
    def rollout_value_hidden(self, x):
        """Critic up to its last hidden pre-activation [n, 256] (the value-fused GAE scan applies the
        activation and the output layer)."""
        rep_outs = self._rep_forward(x)
        s = rep_outs[-1] if rep_outs else x
        lin_ch = self.critic[-2][0]
        return F.linear(s, lin_ch.weight, lin_ch.bias)

    @torch.no_grad()
    def rollout_value_split(self, x, out=None):
        """K40V (r06): the critic from x to its value in two launches — the trunk, then the critic's hidden layer on the
        split GEMM (the rollout's planes of Wh_critic^T, rollout_refresh) with act . w_out + b_out in its epilogue — or
        None where that form does not apply (no rollout planes, a critic deeper than one hidden layer)."""
        rs = getattr(self, "_roll_split", None)
        if rs is None or len(self.critic) != 2:
            return None
        lin_ch, code, slope = self.critic[-2]
        lin_co = self.critic[-1][0]
        if lin_co.out_features != 1 or lin_ch.in_features != 256 or lin_ch.out_features != 256:
            return None
        rep_outs = self._rep_forward(x)
        s = rep_outs[-1] if rep_outs else x
        if not (isinstance(s, torch.Tensor) and s.dim() == 2 and s.shape[1] == 256 and _vec4_rows(s)):
            return None
        return ops.s3_gemm_value(s, rs[1], 256, lin_ch.bias, code, slope, lin_co.weight.view(-1), lin_co.bias, out=out)

    @torch.no_grad()
    def rollout_value(self, x, out=None):
        """Critic only (bootstrap values): trunk, critic hidden GEMM, K14 value head."""
        rep_outs = self._rep_forward(x)
        s = rep_outs[-1] if rep_outs else x
        lin_ch, code, slope = self.critic[-2]
        lin_co = self.critic[-1][0]
        z = F.linear(s, lin_ch.weight, lin_ch.bias)
        return ops.value_head(z, (code, slope), lin_co.weight, lin_co.bias, out=out)

    @torch.no_grad()
    def forward_hidden(self, x, adv=None, adv_partials=None):
        """Forward up to the heads' last hidden pre-activations (K12 does the rest).  x may be Rows(flat, idx); then
        adv_partials (if given) receives the minibatch's advantage moments of adv[idx] (K4's partials)."""
        rep_outs = self._rep_forward(x, adv=adv, adv_partials=adv_partials,
                                     defer_trunk=self.pair is not None and self.gemm_heads)
        s = rep_outs[-1] if rep_outs else x
        if self.pair is not None and self.gemm_heads:   # K16 forms z inside the head kernels
            return (x, rep_outs, s, (([], s, None), ([], s, None)))
        if self.pair is not None:   # one GEMM for both hidden layers: [B, 512] = actor | critic
            H = ops.HEAD_HIDDEN
            ev = ops.TIMER.start("gemm_pair")
            z = F.linear(s, self.pair[0], self.pair[1])
            ops.TIMER.stop("gemm_pair", ev)
            return (x, rep_outs, s, (([], s, z[:, :H]), ([], s, z[:, H:])))
        heads = []
        for layers in (self.actor, self.critic):
            outs = self._chain_forward(layers[:-2], s)
            lin = layers[-2][0]
            x_h = outs[-1] if outs else s
            heads.append((outs, x_h, F.linear(x_h, lin.weight, lin.bias)))
        return (x, rep_outs, s, heads)

    @torch.no_grad()
    def loss_backward(self, ctx, algo, dist, act, adv, ret, old_logp=None, idx=None, adv_partials=None,
                      clip_range=0.2, vf_coef=0.25, ent_coef=0.0):
        """K12 loss + head backward, then the hidden / trunk GEMMs.  Writes every parameter gradient;
        returns the loss-scalars device tensor (ops.OUT_KEYS)."""
        x, rep_outs, s, ((a_outs, a_xh, z_a), (c_outs, c_xh, z_c)) = ctx
        B = s.shape[0]
        lin_ao, _, _ = self.actor[-1]
        lin_ah, a_code, a_slope = self.actor[-2]
        lin_co, _, _ = self.critic[-1]
        lin_ch, c_code, c_slope = self.critic[-2]
        K = lin_ao.out_features
        paired = self.pair is not None
        if self._hws is None or self._hws.batch != B:
            self._hws = ops.HeadWorkspace(B, K, s.device, paired=paired)
        gemm = wh_split = None
        trunk = x.trunk if z_a is None and isinstance(x, Rows) else None
        splits = []   # (matrix, name): every split this update needs, one launch (xpa_s3_split_batch)
        if z_a is None:   # K16
            gemm = (s, (lin_ah.weight, lin_ah.bias), (lin_ch.weight, lin_ch.bias))
            # K16P / K16Q: Wh^T's planes.  With a deferred trunk the planes select K16R, which runs only behind
            # TRUNK_S3R; the use_trunk_heads opt-in (K16X) takes Wh in f32
            if (ops.S3_GEMMS and ops.S3_HEADS in ("s3p", "s3q") and not ops.K16W_ENABLED
                    and (trunk is None or self._s3r_on())):
                splits += [(lin_ah.weight.t(), "s3p_a"), (lin_ch.weight.t(), "s3p_c")]
        crit = (self._crit_plan(x, rep_outs, c_code, B, s.device)
                if paired and z_a is None and trunk is None and wh_split is None and splits else None)
        scales = cs = None
        if paired and len(self.rep) > 0 and self._dx_split_ok(self.pair[0]):
            splits.append((self.pair[0], "dx"))
            if crit is not None:   # K42C: the critic's rows of the dX split scaled by (1 - slope) wc, + cs
                H = ops.HEAD_HIDDEN
                scales = [None] * (len(splits) - 1) + [(lin_co.weight.view(-1), 1.0 - float(c_slope), H)]
                cs = (crit[2], float(c_slope))
        if splits:
            bufs = self._split_many(splits, scales, cs)
            if splits[0][1] == "s3p_a":
                wh_split = (bufs[0], bufs[1])
        grads = {"w_actor": lin_ao.weight.grad, "b_actor": lin_ao.bias.grad, "bh_actor": lin_ah.bias.grad,
                 "w_critic": lin_co.weight.grad, "b_critic": lin_co.bias.grad, "bh_critic": lin_ch.bias.grad}
        if self.logstd is not None:
            grads["logstd"] = self.logstd.grad
        if self._sq is None:
            self._sq = torch.zeros(self.SQ_SLOTS, dtype=torch.float64, device=s.device)
        self.sq_ready = None
        scalars, dz_a, dz_c = ops.fused_heads(algo, dist, self._hws, z_a, lin_ao.weight, lin_ao.bias, (a_code, a_slope),
                                              z_c, lin_co.weight, lin_co.bias, (c_code, c_slope), self.logstd, act,
                                              adv, ret, old_logp=old_logp, idx=idx, adv_partials=adv_partials,
                                              clip_range=clip_range, vf_coef=vf_coef, ent_coef=ent_coef, grads=grads,
                                              colsum_queue=self._cq, gemm=gemm, sq_logstd=self._sq.data_ptr(),
                                              wh_split=wh_split,
                                              defer_loss=True,
                                              trunk=trunk,
                                              crit_mask=crit[:2] if crit is not None else None)
        have_rep = len(self.rep) > 0
        if paired and crit is not None:   # r05: K41P + K42C, the critic's half factored (dz_critic never written)
            q = self._cq_early if self.early_grad_sync is not None else self._cq
            self._weight_grad_pair(s, crit, lin_co, c_slope, q)
            if self.early_grad_sync is not None:
                self._cq_early.flush(s.device)
                self.early_grad_sync(self.pair[2])
            if not self._trunk_bwd_fused(self._hws.dz_actor, x, rep_outs, crit=crit):
                raise RuntimeError("factored critic planned but the fused trunk backward did not apply")
            self._flush_with_norm(s.device)
            return scalars
        if paired:   # dW of both hidden layers and dX (K = 512, no accumulate pass) as single GEMMs
            dz = self._hws.dz_pair
            if self.early_grad_sync is not None:
                # data-parallel: finalize this 0.5 MB slice now and start its all-reduce, which then overlaps
                # the dX GEMM and the trunk backward (distributed.GradAllReduce.begin)
                self._weight_grad(dz, s, self.pair[2], queue=self._cq_early)
                self._cq_early.flush(s.device)
                self.early_grad_sync(self.pair[2])
            else:
                self._weight_grad(dz, s, self.pair[2], queue=self._cq)
            if have_rep and not self._trunk_bwd_fused(dz, x, rep_outs):
                self._chain_backward(self.rep, [x] + rep_outs[:-1], rep_outs, self._dx(dz, self.pair[0]),
                                     need_dx=False, thin_first=self.thin0)
            self._flush_with_norm(s.device)   # every deferred column-sum finalize in one launch
            return scalars
        ds = self._from_dz(self.actor[:-1], [s] + a_outs, a_outs, dz_a, need_dx=have_rep)
        ds = self._from_dz(self.critic[:-1], [s] + c_outs, c_outs, dz_c, need_dx=have_rep, accumulate=ds)
        if have_rep:
            r_in = [x] + rep_outs[:-1]
            self._chain_backward(self.rep, r_in, rep_outs, ds, need_dx=False, thin_first=self.thin0)
        self._flush_with_norm(s.device)
        return scalars

    SQ_SLOTS = 16384   # clip-norm partials: slot 0 = d logstd, then one per finalize column tile

    def _flush_with_norm(self, device):
        """Flush the column-sum finalizes, writing the clip norm's squared-sum partials beside them.  When
        those outputs plus d logstd are every parameter's gradient, sq_ready = (partials, count) lets the
        clip + Adam step skip its norm pass (xpa_clip_adam_step_partials)."""
        total, written = self._cq.flush(device, sq=self._sq)
        covered = written + (self.logstd.numel() if self.logstd is not None else 0)
        if self._n_params is None:
            self._n_params = sum(p.numel() for p in self._params)
        self.sq_ready = (total, 1) if total is not None and covered == self._n_params else None

    def _from_dz(self, layers, inputs, outs, dz, need_dx, accumulate=None):
        """Backward from the pre-activation gradient dz of layers[-1] (its bias gradient already
        written): weight gradient, dX, then the earlier layers of the chain."""
        lin = layers[-1][0]
        self._weight_grad(dz, inputs[len(layers) - 1], lin.weight.grad)
        if len(layers) == 1:
            if not need_dx:
                return None
            return accumulate.addmm_(dz, lin.weight) if accumulate is not None else torch.mm(dz, lin.weight)
        g = torch.mm(dz, lin.weight)
        prev = layers[:-1]
        return self._chain_backward(prev, inputs[:len(prev)], outs[:len(prev)], g, need_dx, accumulate,
                                    allow_head=False)

    # ------------------------------------------------------------------------------------------------
    def _bias_grad(self, code, g, h, slope, out):
        rows, cols = g.shape
        key = (rows, cols)
        part = self._partials.get(key)
        if part is None:
            part = torch.empty((int(ops.lib().xpa_act_bwd_num_partials(rows)), cols), dtype=torch.float32,
                               device=g.device)
            self._partials[key] = part
        s = ops._stream(g.device)
        L = ops.lib()
        _lib.check(L.xpa_act_bwd_colsum(code, ops._p(g), ops._p(h) if code else None, rows, cols, slope,
                                        ops._p(g) if code else None, ops._p(part), s), "xpa_act_bwd_colsum")
        _lib.check(L.xpa_colsum_finalize(ops._p(part), part.shape[0], cols, ops._p(out), s), "xpa_colsum_finalize")

    def _split_buf(self, k, name, device):
        key = ("s3split", name, k)
        buf = self._partials.get(key)
        if buf is None:   # graph-capture safe: allocated on first (eager) use
            buf = torch.empty(int(ops.lib().xpa_s3_split_bytes(k, 256)), dtype=torch.uint8, device=device)
            self._partials[key] = buf
        return buf

    def _split_many(self, items, scales=None, cs=None):
        """The bf16 planes of every (matrix [k, 256], name) in one launch, into buffers kept per name (scales / cs:
        ops.s3_split_batch's, for K42C)."""
        bufs = [self._split_buf(b.shape[0], name + ("_crit" if scales and sc else ""), b.device)
                for (b, name), sc in zip(items, scales or [None] * len(items))]
        ops.s3_split_batch([(b, o) for (b, _), o in zip(items, bufs)], scales, cs)
        return bufs

    # r05: the critic's half of the paired hidden layer's dX and dW factored (K42C / K41P: masked GEMMs on exact 0 / 1
    # operands, three split products instead of six; dz_critic never stored) where it applies: the K16Q heads, a
    # LeakyReLU / ReLU critic hidden layer and K42S's trunk backward
    CRIT_FACTORED = True

    def _crit_plan(self, x, rep_outs, c_code, B, device):
        """(mask int32 [B, 8], dv [B], cs [256]) buffers when the factored critic backward applies, else None."""
        if not (self.CRIT_FACTORED and ops.S3_GEMMS and ops.S3_HEADS == "s3q" and not ops.K16W_ENABLED and c_code == 1
                and self.critic[-1][0].out_features == 1 and self.pair is not None and len(self.rep) == 1):
            return None
        lin, code, _ = self.rep[0]
        if not (self.FUSE_TRUNK_BWD and self._dx_split_ok(self.pair[0]) and code in (0, 1)
                and ((self.thin0 and lin.in_features <= 32) or self._wide_on())
                and isinstance(x, Rows) and getattr(x, "hsign", None) is not None):
            return None
        xr = x.gathered
        h = rep_outs[0] if rep_outs else None
        x_ok = self._wide_on() or (isinstance(xr, torch.Tensor) and xr.dim() == 2 and xr.stride(1) == 1)
        if not (x_ok and isinstance(h, torch.Tensor) and h.shape[1] == 256 and _vec4_rows(h)):
            return None
        if self._hws is None or self._trunk_bwd_form(self._hws.dz_actor, x, rep_outs) is None:
            return None
        key = ("crit", B)
        bufs = self._partials.get(key)
        if bufs is None:   # graph-capture safe: allocated on first (eager) use
            bufs = (torch.empty((B, 8), dtype=torch.int32, device=device), torch.empty((B,), dtype=torch.float32,
                                                                                       device=device),
                    torch.empty((256,), dtype=torch.float32, device=device))
            self._partials[key] = bufs
        return bufs

    def _weight_grad_pair(self, s, crit, lin_co, c_slope, queue):
        """K41P: the paired hidden layer's dW slices (actor: dz_a^T h; critic: factored), two finalize segments."""
        B = s.shape[0]
        sa, per_a, sc, per_c = ops.s3_wgrad_pair_slices(B)
        key = ("wgrad_pair", sa, sc)
        ws = self._partials.get(key)
        if ws is None:
            ws = (torch.empty((sa, 256, 256), dtype=torch.float32, device=s.device),
                  torch.empty((sc, 256, 256), dtype=torch.float32, device=s.device))
            self._partials[key] = ws
        ops.s3_wgrad_pair(self._hws.dz_actor, s, crit[0], crit[1], lin_co.weight.view(-1), c_slope, ws[0], ws[1])
        g = self.pair[2]
        queue.add(ws[0].view(sa, -1), g[:256].reshape(-1))
        queue.add(ws[1].view(sc, -1), g[256:].reshape(-1))

    FUSE_TRUNK_BWD = True   # K42 where it applies (ops.S3_GEMMS, one thin representation layer)
    # K16R where it applies (the split heads, one thin representation layer with the heads' activation): h formed
    # inside both head launches from the gathered rows (K13 only gathers), the actor writes h and its sign bits
    # (r04n: K16R measured slower at C2 — actor 132 / critic 108 us vs K16P's 80 / 63 on h from HBM: the in-loop trunk
    # FMAs are not hidden behind the MFMAs — so it is an opt-in)
    TRUNK_S3R = False
    # K42S by default: K13's gather form writes h's sign bits beside h and K42 reads them instead of h
    SIGN_BITS = True

    def _s3r_on(self):
        return (self.TRUNK_S3R and self.trunk_heads and ops.S3_GEMMS and ops.S3_HEADS in ("s3p", "s3q")
                and not ops.K16W_ENABLED)

    def _sign_on(self, code):
        return (self.SIGN_BITS and self.FUSE_TRUNK_BWD and code in (0, 1) and len(self.rep) == 1 and self.pair is not None
                and self._dx_split_ok(self.pair[0]) and self.rep[0][0].in_features <= 32)

    def _sign_buf(self, B, device):
        key = ("hsign", B)
        sign = self._partials.get(key)
        if sign is None:   # graph-capture safe: allocated on first (eager) use
            sign = torch.empty((B, 8), dtype=torch.int32, device=device)
            self._partials[key] = sign
        return sign

    def _trunk_bwd_form(self, dz, x, rep_outs):
        """Which fused trunk backward applies (no side effects): "wide" (_wide_bwd), "thin" (K42 over K13's layer) or
        None.  _crit_plan plans the factored critic only where this is not None, and _trunk_bwd_fused runs exactly this
        form, so the two cannot disagree."""
        if (self._wide_on() and isinstance(x, Rows) and getattr(x, "hsign", None) is not None
                and (isinstance(x.gathered, torch.Tensor) or getattr(x, "wide_direct", False)) and _vec4_rows(dz)):
            return "wide"
        if not (self.FUSE_TRUNK_BWD and self.pair is not None and self._dx_split_ok(self.pair[0]) and len(self.rep) == 1
                and self.thin0 and _vec4_rows(dz)):
            return None
        xr = x.gathered if isinstance(x, Rows) else x
        if not isinstance(xr, torch.Tensor) or xr.dim() != 2 or xr.stride(1) != 1 or self.rep[0][0].in_features > 32:
            return None
        h = rep_outs[0] if rep_outs else None
        if not isinstance(h, torch.Tensor) or h.stride(1) != 1 or h.shape[1] != 256:
            return None
        return "thin"

    def _trunk_bwd_fused(self, dz, x, rep_outs, crit=None):
        """K42: the dX GEMM and the one representation layer's backward (K13's) in one launch, g never stored.  Returns
        False (nothing done) when it does not apply (_trunk_bwd_form): not the split GEMMs, more than one representation
        layer, no K13 first layer, d_in > 32, or rows not given as the gathered minibatch.  The wide trunk layer:
        _wide_bwd."""
        form = self._trunk_bwd_form(dz, x, rep_outs)
        if form == "wide":
            return self._wide_bwd(dz, x, crit)
        if form is None:
            return False
        lin, code, slope = self.rep[0]
        xr = x.gathered if isinstance(x, Rows) else x
        h = rep_outs[0]
        rows = dz.shape[0]
        key = ("k42", rows, lin.in_features)
        ws = self._partials.get(key)
        if ws is None:
            G = int(ops.lib().xpa_s3_gemm_trunk_bwd_num_partials(rows))
            ws = (torch.empty((G, 256 * lin.in_features), device=dz.device), torch.empty((G, 256), device=dz.device))
            self._partials[key] = ws
        k = self.pair[0].shape[0]
        trunk = getattr(x, "trunk", None) if isinstance(x, Rows) else None
        sign = trunk[5] if trunk is not None and len(trunk) > 5 else None   # K42S: act' from K16R's sign bits
        if sign is None and isinstance(x, Rows):
            sign = getattr(x, "hsign", None)   # or from K13's
        if crit is not None:   # K42C: dz = the actor's half only
            H = ops.HEAD_HIDDEN
            ops.s3_gemm_trunk_bwd_crit(dz, self._split_buf(k, "dx_crit", dz.device), H, k - H, crit[0], crit[1],
                                       crit[2], sign, xr, code, slope, ws[0], ws[1])
        else:
            ops.s3_gemm_trunk_bwd(dz, self._split_buf(k, "dx", dz.device), k, h, xr, code, slope, ws[0], ws[1],
                                  h_sign=sign)
        self._cq.add(ws[0], lin.weight.grad)
        self._cq.add(ws[1], lin.bias.grad)
        return True

    @staticmethod
    def _dx_split_ok(w):
        return ops.S3_GEMMS and w.shape[1] == 256 and w.shape[0] % 16 == 0

    def _dx(self, dz, w):
        """dX = dz w (w [k, n_in]): K40 on the bf16 matrix cores by the three-way split when ops.S3_GEMMS and the shape
        fits (n_in = 256, k % 16 == 0; w's planes were written by this update's split launch), else the f32 GEMM."""
        k, n_in = w.shape
        if not (self._dx_split_ok(w) and _vec4_rows(dz)):
            return torch.mm(dz, w)
        return ops.s3_gemm(dz, self._split_buf(k, "dx", dz.device), k)

    def _weight_grad(self, dz, x, out, queue=None):
        """dW = dz^T x.  Split-K (a batched GEMM over slices of the batch) when the GEMM alone would not
        fill the chip; with `queue` the slice sum is one more segment of the batched column-sum finalize
        (f64, fixed order) instead of its own reduction launch.  With ops.S3_GEMMS and a fitting shape (n_in = 256,
        n_out % 128 == 0) the slices come from K41 on the bf16 matrix cores by the three-way split."""
        B, n_out = dz.shape
        n_in = x.shape[1]
        if (queue is not None and ops.S3_GEMMS and n_in == 256 and n_out % 128 == 0 and isinstance(x, torch.Tensor)
                and _vec4_rows(x) and _vec4_rows(dz)):
            S = ops.s3_wgrad_slices(B, n_out)
            key = ("s3wgrad", S, n_out)
            ws = self._partials.get(key)
            if ws is None:
                ws = torch.empty((S, n_out, n_in), dtype=torch.float32, device=dz.device)
                self._partials[key] = ws
            ops.s3_wgrad(dz, x, out=ws)
            queue.add(ws.view(S, n_out * n_in), out.view(-1))
            return
        s = _splitk_splits(B, n_out, n_in)
        if queue is not None:   # (s == 1: the finalize only copies, so every gradient still passes through it)
            key = ("splitk", s, n_out, n_in)
            ws = self._partials.get(key)
            if ws is None:
                ws = torch.empty((s, n_out, n_in), dtype=torch.float32, device=dz.device)
                self._partials[key] = ws
            if s > 1:
                torch.bmm(dz.view(s, B // s, n_out).transpose(1, 2), x.reshape(s, B // s, n_in), out=ws)
            else:
                torch.mm(dz.t(), x, out=ws[0])
            queue.add(ws.view(s, n_out * n_in), out.view(-1))
            return
        if s > 1:
            torch.sum(torch.bmm(dz.view(s, B // s, n_out).transpose(1, 2), x.reshape(s, B // s, n_in)), dim=0,
                      out=out)
        else:
            torch.mm(dz.t(), x, out=out)

    def _head_tail(self, layers, outs, g):
        """K11 for [hidden Linear + act] -> [output Linear, no act]: returns dz of the hidden layer."""
        lin_o, code_o, _ = layers[-1]
        lin_h, code_h, slope = layers[-2]
        h = outs[-2]
        B, H = h.shape
        K = g.shape[1]
        key = ("head", B, H, K)
        ws = self._partials.get(key)
        L = ops.lib()
        if ws is None:
            G = int(L.xpa_head_bwd_num_partials(B))
            dev = g.device
            ws = (torch.empty((G, K * H), device=dev), torch.empty((G, H), device=dev), torch.empty((G, K), device=dev),
                  torch.empty((B, H), device=dev))
            self._partials[key] = ws
        p_dw, p_dbh, p_dbo, dz = ws
        s = ops._stream(g.device)
        _lib.check(L.xpa_head_backward(code_h, K, ops._p(g), g.stride(0), ops._p(h), ops._p(lin_o.weight), B, H, slope,
                                       ops._p(dz), ops._p(p_dw), ops._p(p_dbh), ops._p(p_dbo), s), "xpa_head_backward")
        G = p_dw.shape[0]
        _lib.check(L.xpa_colsum_finalize(ops._p(p_dw), G, K * H, ops._p(lin_o.weight.grad), s), "colsum dW")
        _lib.check(L.xpa_colsum_finalize(ops._p(p_dbh), G, H, ops._p(lin_h.bias.grad), s), "colsum db_h")
        _lib.check(L.xpa_colsum_finalize(ops._p(p_dbo), G, K, ops._p(lin_o.bias.grad), s), "colsum db_o")
        return dz

    def _chain_backward(self, layers, inputs, outs, g, need_dx, accumulate=None, allow_head=True, thin_first=False):
        """g: grad w.r.t. the chain's last output (contiguous [B, n_out]); returns grad w.r.t. its input
        (added to `accumulate` through the GEMM's C operand when given)."""
        top = len(layers) - 1
        if (len(layers) >= 2 and layers[-1][1] == 0 and layers[-2][1] != 0 and g.shape[1] <= 32
                and g.stride(1) == 1 and self.use_head_kernel and allow_head):
            g = self._head_tail(layers, outs, g)   # output layer + hidden activation done by K11
            lin, _, _ = layers[-2]
            self._weight_grad(g, inputs[-2], lin.weight.grad)
            top = len(layers) - 2
            if top > 0 or need_dx:
                if top == 0 and accumulate is not None:
                    g = accumulate.addmm_(g, lin.weight)
                else:
                    g = torch.mm(g, lin.weight)
            top -= 1
        for j in range(top, -1, -1):
            lin, code, slope = layers[j]
            h = outs[j]
            x = inputs[j]
            if j == 0 and thin_first and not need_dx and g.stride(1) == 1 and (isinstance(x, Rows) or x.stride(1) == 1):
                self._thin_backward(layers[0], g, h, x)   # K13: act backward + dW + db, no dz pass
                break
            self._bias_grad(code, g, h, slope, lin.bias.grad)   # g <- g * act'(h) in place (code != 0)
            self._weight_grad(g, x, lin.weight.grad)
            if j > 0 or need_dx:
                if j == 0 and accumulate is not None:
                    g = accumulate.addmm_(g, lin.weight)   # C += g W in the GEMM (C aliases D: no copy)
                else:
                    g = torch.mm(g, lin.weight)
        return g

    @torch.no_grad()
    def backward(self, ctx, d_head, d_v):
        x, rep_outs, s, a_outs, c_outs = ctx
        have_rep = len(self.rep) > 0
        a_in = [s] + a_outs[:-1]
        c_in = [s] + c_outs[:-1]
        ds = self._chain_backward(self.actor, a_in, a_outs, d_head, need_dx=have_rep)
        ds = self._chain_backward(self.critic, c_in, c_outs, d_v.view(-1, 1), need_dx=have_rep, accumulate=ds)
        if have_rep:
            r_in = [x] + rep_outs[:-1]
            self._chain_backward(self.rep, r_in, rep_outs, ds, need_dx=False, thin_first=self.thin0)
        self._cq.flush(d_head.device)
