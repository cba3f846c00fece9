"""Explicit (autograd-free) forward / backward of the convolutional policies: the AC_CNN_Atari actor-critic (C3) and
the Basic_CNN Q-network of PER-DQN (C5).

Reference: AC_CNN_Atari xuance/torch/representations/cnn.py:45-93 (conv blocks with padding (k - s) // 2 + ReLU,
Flatten, fc blocks), Basic_CNN cnn.py:5-40 (conv blocks, AdaptiveMaxPool2d((1, 1)), Flatten), cnn_block / mlp_block
xuance/torch/utils/layers.py:8-57, Categorical_AC_Policy xuance/torch/policies/categorical.py:61-85, BasicQnetwork
deterministic.py:148-182; the learners' loss.backward() (a2c_learner.py:31-33, perdqn_learner.py:37-40).

Every activation stays NHWC ([rows = B*H*W, C] row-major), the layout the uint8 frames arrive in:
  forward   the first conv block: K25 xpa_conv1_u8_fwd (the 4 x 8 x 8 -> 32 conv on fp32 MFMA straight from the uint8
            frames as sum x (w / 255) — one f32 rounding per term like the reference's sum float(x / 255) w —, bias
            + ReLU in its epilogue); other first layers: K20 xpa_frames_to_f32 then MIOpen as below
            -> per conv: MIOpen conv2d without bias on the channels-last view -> K21 xpa_bias_act (bias + ReLU
               in place)
            -> AC_CNN_Atari: Flatten in NHWC order — the first fc layer uses its weight with the columns permuted
               from the reference's (C, H, W) order to (H, W, C) (one 13 MB copy per parameter update, instead of an
               NHWC -> NCHW copy of the [B, 6400] activations every forward) -> fc: hipBLASLt GEMM (bias epilogue)
               -> K21 ReLU in place;
               Basic_CNN: K23 xpa_global_maxpool (max + argmax per (b, c), torch's tie rule)
            -> heads / Q head (GEMMs)
  backward  heads: GEMMs + K10 / K22 bias column sums -> AC_CNN_Atari fc: K22 xpa_act_bwd_bias (ReLU backward + bias
            gradient) -> dW GEMM (permuted back into the reference layout) + dX GEMM; Basic_CNN: K24 (the pooled
            gradient routed to the argmax, ReLU backward, bias gradient) -> per conv: K22 then MIOpen
            convolution_backward (weight; data too except where K27 xpa_conv_dgrad_s2k takes the data gradient — the
            4 x 4 stride-2 32 -> 64 conv); the first conv (no dX) after K25: K26 xpa_conv1_u8_wgrad_act from the uint8
            frames with its ReLU backward + bias gradient folded in (no K22 pass) + the f64 column-sum finalizes (no
            f32 frame copy anywhere).
Parameter gradients are written into the parameters' .grad views (allocated when missing).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib, ops
from .fused_mlp import _act_code, _parse
from .policies import AC_CNN_Atari, Basic_CNN, policy_discrete


def _conv_layers(model):
    """(conv blocks [(conv, act code, slope)], tail, fc layers): tail "flatten" (AC_CNN_Atari) or "maxpool"
    (Basic_CNN)."""
    convs, i = [], 0
    mods = list(model)
    while i < len(mods) and isinstance(mods[i], nn.Conv2d):
        conv = mods[i]
        nxt = mods[i + 1] if i + 1 < len(mods) else None
        act = nxt if isinstance(nxt, (nn.ReLU, nn.LeakyReLU, nn.Tanh)) else None
        if conv.bias is None or conv.groups != 1 or tuple(conv.dilation) != (1, 1):
            raise ValueError("expected Conv2d with bias, groups 1, dilation 1")
        convs.append((conv,) + _act_code(act))
        i += 2 if act is not None else 1
    if not convs:
        raise ValueError("no conv blocks")
    if i < len(mods) and isinstance(mods[i], nn.AdaptiveMaxPool2d):
        if tuple(nn.modules.utils._pair(mods[i].output_size)) != (1, 1) or i + 1 >= len(mods) \
                or not isinstance(mods[i + 1], nn.Flatten) or i + 2 != len(mods):
            raise ValueError("expected AdaptiveMaxPool2d((1, 1)) + Flatten as the tail")
        return convs, "maxpool", []
    if i >= len(mods) or not isinstance(mods[i], nn.Flatten):
        raise ValueError("expected Flatten (or a global max pool) after the conv blocks")
    fc = _parse(mods[i + 1:])
    if not fc:
        raise ValueError("Flatten without fc layers")
    return convs, "flatten", fc


class _Part:
    """Per-block partial buffers of the bias-gradient reductions, by shape."""

    def __init__(self):
        self.bufs = {}

    def buf(self, key, shape, device):
        """A cached float32 buffer by key (K28 / K29 partials)."""
        p = self.bufs.get(key)
        if p is None:
            p = torch.empty(shape, dtype=torch.float32, device=device)
            self.bufs[key] = p
        return p

    def get(self, rows, cols, device, k22):
        key = (rows, cols, k22)
        p = self.bufs.get(key)
        if p is None:
            L = ops.lib()
            G = int(L.xpa_act_bwd_bias_num_partials(rows, cols)) if k22 else int(L.xpa_act_bwd_num_partials(rows))
            p = torch.empty((G, cols), dtype=torch.float32, device=device)
            self.bufs[key] = p
        return p


def _bias_act(code, y2d, bias, slope):
    _lib.check(ops.lib().xpa_bias_act(code, ops._p(y2d), y2d.shape[0], y2d.shape[1],
                                      ops._p(bias) if bias is not None else None, float(slope),
                                      ops._stream(y2d.device)), "xpa_bias_act")


def _act_bwd_bias(parts, code, g2d, h2d, slope, bias_grad):
    """g2d <- g2d * act'(h2d) in place; bias_grad <- column sums (K22, or K10 for widths K22 does not take)."""
    rows, cols = g2d.shape
    L, s = ops.lib(), ops._stream(g2d.device)
    if not g2d.is_contiguous():
        raise ValueError("gradient rows must be contiguous")
    k22 = cols % 4 == 0 and 256 % (cols // 4) == 0
    part = parts.get(rows, cols, g2d.device, k22)
    hp = ops._p(h2d) if code else None
    gp = ops._p(g2d) if code else None
    if k22:
        _lib.check(L.xpa_act_bwd_bias(code, ops._p(g2d), hp, rows, cols, float(slope), gp, ops._p(part), s),
                   "xpa_act_bwd_bias")
    else:
        _lib.check(L.xpa_act_bwd_colsum(code, ops._p(g2d), hp, rows, cols, float(slope), gp, ops._p(part), s),
                   "xpa_act_bwd_colsum")
    _lib.check(L.xpa_colsum_finalize(ops._p(part), part.shape[0], cols, ops._p(bias_grad), s), "xpa_colsum_finalize")


def _chain(layers, x):
    outs, h = [], x
    for lin, code, slope in layers:
        h = F.linear(h, lin.weight, lin.bias)
        if code and h.shape[1] % 4 == 0 and 256 % (h.shape[1] // 4) == 0:
            _bias_act(code, h, None, slope)   # K21 in place
        elif code == 1:
            F.leaky_relu(h, slope, inplace=True)
        elif code == 2:
            h.tanh_()
        outs.append(h)
    return outs


def _chain_backward(parts, layers, inputs, outs, g, acc=None, need_dx=True):
    """Linear(+act) chain backward; returns d(input) (added into acc when given)."""
    for j in range(len(layers) - 1, -1, -1):
        lin, code, slope = layers[j]
        g = g.contiguous()
        _act_bwd_bias(parts, code, g, outs[j], slope, lin.bias.grad)
        torch.mm(g.t(), inputs[j], out=lin.weight.grad)
        if j == 0 and not need_dx:
            return None
        if j == 0 and acc is not None:
            g = acc.addmm_(g, lin.weight)
        else:
            g = torch.mm(g, lin.weight)
    return g


def _library_conv_guard(conv):
    """The explicit CNN path refuses MIOpen for convolutions with fewer than 16 input or output channels.  The r02
    intermittent hipErrorIllegalAddress of the PER-DQN agent loop (2 of 9 runs, 8-channel test net)
    surfaced at the first host sync after one agent step whose only library convolutions were MIOpen's NHWC kernels
    for 4 / 8-channel shapes; every hand-written kernel of that step carries a device error word since r03 and
    reported 0 in every later run.  K28 / K29 take every such conv, so reaching MIOpen here means use_igemm was turned
    off (or a shape K28 / K29 reject): an error instead of the unproven route."""
    if min(conv.in_channels, conv.out_channels) < 16:
        raise RuntimeError("conv %d -> %d channels: the small-channel MIOpen route is refused (r02 fault suspect); "
                           "keep use_igemm on (K28 / K29 take convs with in_channels %% 4 == 0, <= 64 channels)"
                           % (conv.in_channels, conv.out_channels))


def _ensure_grads(params):
    for p in params:
        if p.grad is None:
            p.grad = torch.zeros_like(p)


class _Trunk:
    """The explicit forward / backward of one AC_CNN_Atari or Basic_CNN representation."""

    def __init__(self, rep, parts):
        # structural, not nominal: the reference's own AC_CNN_Atari / Basic_CNN (cnn.py:5-93: a `.model` nn.Sequential
        # of conv blocks [+ max pool] + Flatten [+ fc blocks], input_shape (C, H, W), observations / 255 in forward)
        # take this path as ours do; _conv_layers raises ValueError on anything else
        if not (isinstance(rep, (AC_CNN_Atari, Basic_CNN)) or (isinstance(getattr(rep, "model", None), nn.Sequential)
                                                                and len(getattr(rep, "input_shape", ())) == 3)):
            raise ValueError("representation %r has no explicit CNN path" % type(rep).__name__)
        self.rep = rep
        self.convs, self.tail, self.fc = _conv_layers(rep.model)
        for conv, _, _ in self.convs:
            if conv.out_channels % 4 or 256 % (conv.out_channels // 4):
                raise ValueError("conv channels must be a multiple of 4 dividing 1024")
        C, H, W = rep.input_shape
        self.in_hwc = (H, W, C)
        shape = (C, H, W)
        for conv, _, _ in self.convs:
            k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
            shape = (conv.out_channels, (shape[1] + 2 * p - k) // s + 1, (shape[2] + 2 * p - k) // s + 1)
        self._chw = shape
        if self.tail == "flatten" and self.fc[0][0].in_features != shape[0] * shape[1] * shape[2]:
            raise ValueError("fc input width does not match the conv output")
        self._w_hwc = None      # the first fc weight with (H, W, C)-ordered columns, refreshed after each update
        self._w_ver = 0         # bumped whenever _w_hwc is re-derived (the fc split planes follow it)
        self._fcs = None        # K40G planes of _w_hwc (forward k halves, data-gradient column blocks) + their version
        self.stale = True
        self._dw_tmp = None
        self.parts = parts
        self.n_params = 2 * (len(self.convs) + len(self.fc))
        # K25: the first conv block straight from the uint8 frames (4 channels, 8 x 8 kernel, 32 outputs: the Nature
        # CNN's first layer); the f32 frame copy (K20) is then only made in the backward, for MIOpen's weight gradient
        c0 = self.convs[0][0]
        self.u8_conv1 = (C == 4 and c0.in_channels == 4 and c0.out_channels == 32 and tuple(c0.kernel_size) == (8, 8)
                         and c0.stride[0] == c0.stride[1] and c0.padding[0] == c0.padding[1]
                         and c0.padding_mode == "zeros")
        # a small-channel conv (< 16 in or out) must run on K28 / K29 (forward, weight gradient and, past the first
        # block, the data gradient): MIOpen's small-channel route is refused (_library_conv_guard).  A net with such
        # a conv that K28 / K29 cannot take (e.g. a 3-channel RGB first conv, in_channels % 4 != 0) gets no explicit
        # path: ValueError here sends the learner to the generic autograd path instead of failing mid-update.
        for i, (conv, _, _) in enumerate(self.convs):
            if min(conv.in_channels, conv.out_channels) >= 16 or (i == 0 and self.u8_conv1):
                continue
            if not self._igemm_shape_ok(conv) or (i > 0 and not self._dgrad_ok(conv)
                                                  and not self._igemm_dgrad_shape_ok(conv)):
                raise ValueError("conv %d -> %d channels (kernel %s): no K28 / K29 form and the small-channel "
                                 "library route is refused" % (conv.in_channels, conv.out_channels,
                                                              tuple(conv.kernel_size)))

    def params(self):
        out = []
        for conv, _, _ in self.convs:
            out += [conv.weight, conv.bias]
        for lin, _, _ in self.fc:
            out += [lin.weight, lin.bias]
        return out

    def refresh(self):
        self.stale = True
        if self.tail == "flatten":
            self._fc0_weight()

    def _fc0_weight(self):
        if self.stale or self._w_hwc is None:
            w = self.fc[0][0].weight
            Cl, Hl, Wl = self._chw
            if self._w_hwc is None:
                self._w_hwc = torch.empty_like(w)
            self._w_hwc.view(w.shape[0], Hl, Wl, Cl).copy_(w.view(w.shape[0], Cl, Hl, Wl).permute(0, 2, 3, 1))
            self.stale = False
            self._w_ver += 1
        return self._w_hwc

    # r05: the first fc layer of the update's minibatches (C3: [16384, 6400] x [6400, 512]) on the bf16 matrix cores by
    # the three-way split (K40G: one launch per GEMM; forward in 2 k halves x 256-column blocks, summed in a fixed
    # order; the data gradient in 256-column blocks, the last one aligned to the end so no block is padded — the
    # columns it shares with its neighbour come out bit-identical from both).  The rollout's 1024-frame forwards stay
    # on hipBLASLt (fc_split_min_rows).  The weight gradient stays on hipBLASLt.
    fc_split = True
    fc_split_min_rows = 8192

    def _fc_split_ok(self, rows):
        if not (self.fc_split and ops.S3_GEMMS and self.tail == "flatten" and rows >= self.fc_split_min_rows):
            return False
        lin = self.fc[0][0]
        return lin.out_features % 256 == 0 and lin.in_features % 32 == 0 and lin.in_features >= 512 and \
            lin.out_features // 256 * 2 <= 32 and (lin.in_features + 255) // 256 <= 32

    def _fc_planes(self):
        """The split planes of the current _w_hwc: forward (column block j, k half p) and data-gradient column
        blocks, re-split (4 matrices per launch) whenever _w_hwc was re-derived."""
        w = self._fc0_weight()
        if self._fcs is not None and self._fcs[0] == self._w_ver:
            return self._fcs
        out_f, in_f = w.shape
        kh = in_f // 2
        fwd = [w[j * 256:(j + 1) * 256, p * kh:(p + 1) * kh].t() for j in range(out_f // 256) for p in range(2)]
        c0s = [min(c, in_f - 256) for c in range(0, in_f, 256)]
        dgr = [w[:, c0:c0 + 256] for c0 in c0s]
        old = self._fcs
        if old is None:
            nb_f, nb_d = int(ops.lib().xpa_s3_split_bytes(kh, 256)), int(ops.lib().xpa_s3_split_bytes(out_f, 256))
            bufs_f = [torch.empty(nb_f, dtype=torch.uint8, device=w.device) for _ in fwd]
            bufs_d = [torch.empty(nb_d, dtype=torch.uint8, device=w.device) for _ in dgr]
        else:
            bufs_f, bufs_d = old[1], old[2]
        pairs = list(zip(fwd, bufs_f)) + list(zip(dgr, bufs_d))
        for i in range(0, len(pairs), 4):
            ops.s3_split_batch(pairs[i:i + 4])
        self._fcs = (self._w_ver, bufs_f, bufs_d, c0s)
        return self._fcs

    def _fc0_forward_split(self, flat, lin, code, slope):
        rows, in_f = flat.shape
        out_f, kh = lin.out_features, in_f // 2
        _, bf, _, _ = self._fc_planes()
        part = self.parts.buf(("fcs", rows, out_f), (2, rows, out_f), flat.device)
        probs = [(flat[:, p * kh:(p + 1) * kh], bf[j * 2 + p], part[p, :, j * 256:(j + 1) * 256])
                 for j in range(out_f // 256) for p in range(2)]
        ops.s3_gemm_group(probs, kh)
        s = torch.add(part[0], part[1])
        _bias_act(code, s, lin.bias, slope)
        return s

    # r05: with the fc split, the data gradient's epilogue also applies the last conv block's activation backward and
    # writes its bias-gradient partials (xpa_s3_gemm_group_act): that block's K22 pass over [B x H x W, C] is gone
    fc_fuse_act = True

    def _fc_fuse_ok(self, rows):
        conv, code, _ = self.convs[-1]
        in_f = self.fc[0][0].in_features
        return (self.fc_fuse_act and self._fc_split_ok(rows) and in_f % 256 == 0 and conv.out_channels in (32, 64)
                and code in (0, 1, 2))

    def _fc0_dgrad_split_act(self, g, y_flat):
        """dz of the last conv block (its output gradient x act'(its output)) from the fc's K40G data gradient, and
        that block's bias gradient (f64 finalize of the per-block partials)."""
        rows = g.shape[0]
        _, _, bd, c0s = self._fc_planes()
        conv, code, slope = self.convs[-1]
        C = conv.out_channels
        dz = torch.empty((rows, self.fc[0][0].in_features), dtype=torch.float32, device=g.device)
        G = int(ops.lib().xpa_s3_gemm_group_act_num_partials(len(c0s), rows))
        part = self.parts.buf(("fcab", rows, C), (G, C), g.device)
        ops.s3_gemm_group_act([(g, b, dz[:, c0:c0 + 256]) for b, c0 in zip(bd, c0s)], g.shape[1],
                              [y_flat[:, c0:c0 + 256] for c0 in c0s], code, slope, C, part)
        _lib.check(ops.lib().xpa_colsum_finalize(ops._p(part), G, C, ops._p(conv.bias.grad), ops._stream(g.device)),
                   "colsum db (fc act)")
        return dz

    # r06: the first fc layer's weight gradient on the split too (was hipBLASLt's f32 GEMM: 822 us per C3 minibatch,
    # profiles/r05/r05k28b): dW^T = flat^T g as K41V slices per 256-column half of g (AC_CNN_Atari: flat [B, 6400] =
    # 50 row tiles of 128; a width that is not a multiple of 128 takes the padded form, the columns past a row reading
    # the next row or the slack the forward leaves after the last row, into output rows the finalize map drops); the
    # batched f64 finalize writes the kept rows transposed into dW.  Same row rule as the forward's split
    # (fc_split_min_rows).
    fc_wsplit = True

    def _fc_wsplit_rows(self, rows):
        lin = self.fc[0][0] if self.fc else None
        return (self.fc_wsplit and lin is not None and ops.S3_GEMMS and self.tail == "flatten"
                and rows >= self.fc_split_min_rows and lin.out_features % 256 == 0 and lin.in_features % 4 == 0)

    def _fc0_wgrad_split(self, g, flat):
        """self._dw_tmp = g^T flat ([out, in], the forward's (H, W, C) column order) on K41V; False (nothing done) where it
        does not apply."""
        rows, in_f = flat.shape
        m = (in_f + 127) // 128 * 128
        if not (self._fc_wsplit_rows(rows) and g.is_contiguous() and flat.stride(1) == 1 and flat.stride(0) == in_f
                and flat.untyped_storage().nbytes() // 4 >= flat.storage_offset() + (rows - 1) * in_f + m):
            return False
        out_f = g.shape[1]
        S = ops.s3_wgrad_slices(rows, m)
        if getattr(self, "_fcq", None) is None:
            self._fcq = ops.ColsumQueue()
        for h in range(out_f // 256):
            part = self.parts.buf(("fcw", h, S, m), (S, m, 256), g.device)
            ops.s3_wgrad(flat, g[:, 256 * h:256 * (h + 1)], out=part, slices=S, m=m if m != in_f else None)
            self._fcq.add(part.view(S, -1), self._dw_tmp[256 * h:256 * (h + 1)], tmap=(256, in_f, in_f))
        self._fcq.flush(g.device)
        return True

    def _fc0_dgrad_split(self, g):
        rows = g.shape[0]
        _, _, bd, c0s = self._fc_planes()
        in_f = self.fc[0][0].in_features
        dx = torch.empty((rows, in_f), dtype=torch.float32, device=g.device)
        ops.s3_gemm_group([(g, b, dx[:, c0:c0 + 256]) for b, c0 in zip(bd, c0s)], g.shape[1])
        return dx

    @staticmethod
    def frames(x):
        """uint8 [B, H, W, C] -> float32 / 255 [B, H, W, C] (K20)."""
        if x.dtype != torch.uint8 or x.device.type != "cuda" or not x.is_contiguous():
            raise ValueError("frames must be a contiguous uint8 ROCm tensor [B, H, W, C]")
        out = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        _lib.check(ops.lib().xpa_frames_to_f32(ops._p(x), x.numel(), ops._p(out), ops._stream(x.device)),
                   "xpa_frames_to_f32")
        return out

    def _conv1_u8(self, xu):
        """K25: act(conv1(x / 255) + b) from the uint8 frames xu [B, H, W, 4] -> NHWC f32."""
        conv, code, slope = self.convs[0]
        B, H, W, C = xu.shape
        k, st, pd = 8, conv.stride[0], conv.padding[0]
        OH, OW = (H + 2 * pd - k) // st + 1, (W + 2 * pd - k) // st + 1
        w = conv.weight if conv.weight.is_contiguous() else conv.weight.contiguous()
        y = torch.empty((B, OH, OW, 32), dtype=torch.float32, device=xu.device)
        _lib.check(ops.lib().xpa_conv1_u8_fwd(code, ops._p(xu), B, H, W, C, k, st, pd, ops._p(w), ops._p(conv.bias), 32,
                                              float(slope), ops._p(y), ops._stream(xu.device)), "xpa_conv1_u8_fwd")
        return y

    @torch.no_grad()
    def forward(self, x):
        """x uint8 [B, H, W, C] -> (state [B, d], context for backward).  With K25 the context keeps the uint8 frames
        as its first entry (backward converts them for the first conv's weight gradient)."""
        B = x.shape[0]
        xu = x.reshape((B,) + self.in_hwc)
        if self.u8_conv1 and xu.dtype == torch.uint8 and xu.is_contiguous() and xu.device.type == "cuda":
            h = self._conv1_u8(xu)
            hs = [xu, h]
            convs = self.convs[1:]
        else:
            h = self.frames(xu)
            hs = [h]
            convs = self.convs
        last = convs[-1][0] if convs else None
        for conv, code, slope in convs:
            if self._igemm_ok(conv, h.numel(), self._out_rows(conv, h.shape)):   # K28 (bias + activation fused)
                # r06: the last block's output (the fc layer's flat input) with slack after it where the split weight
                # gradient will read it as 128-row tiles (_fc0_wgrad_split)
                slack = 0
                if conv is last and self.tail == "flatten" and self._fc_wsplit_rows(B):
                    oh = (h.shape[1] + 2 * conv.padding[0] - conv.kernel_size[0]) // conv.stride[0] + 1
                    ow = (h.shape[2] + 2 * conv.padding[0] - conv.kernel_size[0]) // conv.stride[0] + 1
                    width = oh * ow * conv.out_channels
                    slack = (width + 127) // 128 * 128 - width   # 0 for AC_CNN_Atari's 10 x 10 x 64 = 6400
                y = self._conv_fwd(conv, code, slope, h, slack=slack)
            else:
                _library_conv_guard(conv)
                z = F.conv2d(h.permute(0, 3, 1, 2), conv.weight, None, conv.stride, conv.padding)
                y = z.permute(0, 2, 3, 1)
                if not y.is_contiguous():
                    y = y.contiguous()
                _bias_act(code, y.view(-1, y.shape[3]), conv.bias, slope)
            hs.append(y)
            h = y
        if self.tail == "maxpool":
            Cl = h.shape[3]
            s = torch.empty((B, Cl), dtype=torch.float32, device=x.device)
            am = torch.empty((B, Cl), dtype=torch.int32, device=x.device)
            _lib.check(ops.lib().xpa_global_maxpool(ops._p(h), B, h.shape[1] * h.shape[2], Cl, ops._p(s), ops._p(am),
                                                    ops._stream(x.device)), "xpa_global_maxpool")
            return s, (hs, am, None, [])
        flat = h.reshape(B, -1)                  # (H, W, C) order: no copy
        fouts = []
        s = flat
        for j, (lin, code, slope) in enumerate(self.fc):
            if j == 0 and self._fc_split_ok(B) and flat.is_contiguous():
                s = self._fc0_forward_split(flat, lin, code, slope)
            else:
                w = self._fc0_weight() if j == 0 else lin.weight
                s = F.linear(s, w, lin.bias)
                if code:
                    _bias_act(code, s, None, slope)
            fouts.append(s)
        return s, (hs, None, flat, fouts)

    use_igemm = True   # K28 / K29 for the convs they take (False: MIOpen for every conv, the r02 path)
    # K28 / K29 hold one weight image per CU and tile the output rows 32 at a time per wave, so below ~1 M output rows
    # a launch has too few tiles per CU to balance (C5's batch 2048 = 800 rows per CU = 25 tiles over 16 waves) and
    # MIOpen's kernels measure faster there (tools/c5_ab.py: 2.26 vs 2.65 ms per C5 learner step; C3's rollout
    # forwards at 1024 frames 71 vs 84-94 us).  Small-channel convs (< 16 in or out: the test nets, r02's fault
    # suspect) always take K28 / K29.
    igemm_min_rows = 1 << 20

    @staticmethod
    def _igemm_shape_ok(conv):
        """The shape part of K28 / K29's conditions (no size preference, no 2 GiB operand check)."""
        k, st, pd = conv.kernel_size, conv.stride, conv.padding
        return (k[0] == k[1] and st[0] == st[1] and pd[0] == pd[1] and conv.padding_mode == "zeros"
                and conv.in_channels % 4 == 0 and conv.weight.is_contiguous()
                and bool(ops.lib().xpa_conv_igemm_ok(conv.in_channels, conv.out_channels, k[0])))

    @classmethod
    def _igemm_dgrad_shape_ok(cls, conv):
        k, st = conv.kernel_size, conv.stride
        return (cls._igemm_shape_ok(conv) and st[0] <= 2 and conv.out_channels % 4 == 0
                and bool(ops.lib().xpa_conv_igemm_ok(conv.out_channels, conv.in_channels, k[0])))

    def _igemm_ok(self, conv, numel, rows=None):
        """numel: the largest operand K28 / K29 load (32-bit buffer offsets: under 2 GiB); rows: the conv's output
        pixels B x OH x OW (None: no size preference)."""
        small_c = min(conv.in_channels, conv.out_channels) < 16
        return (self.use_igemm and numel * 4 < 2 ** 31 and (rows is None or small_c or rows >= self.igemm_min_rows)
                and self._igemm_shape_ok(conv))

    def _igemm_dgrad_ok(self, conv, numel, rows=None):
        return self._igemm_ok(conv, numel, rows) and self._igemm_dgrad_shape_ok(conv)

    @staticmethod
    def _out_rows(conv, shape):
        B, H, W = shape[0], shape[1], shape[2]
        k, st, pd = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        return B * ((H + 2 * pd - k) // st + 1) * ((W + 2 * pd - k) // st + 1)

    @staticmethod
    def _conv_fwd(conv, code, slope, h, slack=0):
        """K28 forward: act(conv(h) + b), h NHWC f32 [B, H, W, C] -> NHWC [B, OH, OW, out].  slack: floats of the same
        allocation after the output (readable, never written: the padded K41 reads them into output rows it drops)."""
        B, H, W, C = h.shape
        k, st, pd = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        OH, OW = (H + 2 * pd - k) // st + 1, (W + 2 * pd - k) // st + 1
        h = h if h.is_contiguous() else h.contiguous()
        n = B * OH * OW * conv.out_channels
        y = torch.empty((n + slack,), dtype=torch.float32, device=h.device)[:n].view(B, OH, OW, conv.out_channels)
        _lib.check(ops.lib().xpa_conv_fwd(code, ops._p(h), B, H, W, C, ops._p(conv.weight), ops._p(conv.bias),
                                          conv.out_channels, k, st, pd, float(slope), ops._p(y), ops._stream(h.device)),
                   "xpa_conv_fwd")
        return y

    def _conv_wgrad(self, conv, g, act, slope, y, x):
        """K29: conv.weight.grad (and with act >= 0: g * act'(y) is the operand and conv.bias.grad is written too) from
        g NHWC [B, OH, OW, out] and the block's input x NHWC f32 [B, H, W, in]."""
        L, st = ops.lib(), ops._stream(g.device)
        B, H, W, C = x.shape
        k = conv.kernel_size[0]
        cout, cols = conv.out_channels, k * k * C
        G = int(L.xpa_conv_wgrad_num_partials())
        part = self.parts.buf(("wg", cout, cols), (G, cout * cols), g.device)
        bpart = self.parts.buf(("wgb", cout), (G, cout), g.device) if act >= 0 else None
        g = g if g.is_contiguous() else g.contiguous()
        _lib.check(L.xpa_conv_wgrad(act, ops._p(g), ops._p(y) if act >= 0 else None, float(slope), ops._p(x), B, H, W, C,
                                    cout, k, conv.stride[0], conv.padding[0], ops._p(part), ops._p(bpart), st),
                   "xpa_conv_wgrad")
        _lib.check(L.xpa_colsum_finalize(ops._p(part), G, cout * cols, ops._p(conv.weight.grad), st), "colsum dW")
        if act >= 0:
            _lib.check(L.xpa_colsum_finalize(ops._p(bpart), G, cout, ops._p(conv.bias.grad), st), "colsum db")

    def _conv_dgrad(self, conv, dz, x_shape, prev):
        """K28 data gradient from dz (the block's pre-activation gradient, NHWC) into the block's input; prev = (code,
        slope, y_prev, bias_grad_prev) of the previous block: its activation backward and bias gradient fused in (the
        result is then that block's dz)."""
        L, st = ops.lib(), ops._stream(dz.device)
        B, H, W, Cin = x_shape
        k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        OH, OW = dz.shape[1], dz.shape[2]
        dx = torch.empty((B, H, W, Cin), dtype=torch.float32, device=dz.device)
        code, slope, y_prev, bgrad = prev
        G = int(L.xpa_conv_dgrad_num_partials(B, H, W))
        bpart = self.parts.buf(("dgb", B * H * W, Cin), (G, Cin), dz.device)
        dz = dz if dz.is_contiguous() else dz.contiguous()
        _lib.check(L.xpa_conv_dgrad(ops._p(dz), B, OH, OW, conv.out_channels, ops._p(conv.weight), Cin, k, s, p, H, W,
                                    code, ops._p(y_prev), float(slope), ops._p(dx), ops._p(bpart), st), "xpa_conv_dgrad")
        _lib.check(L.xpa_colsum_finalize(ops._p(bpart), G, Cin, ops._p(bgrad), st), "colsum db (dgrad)")
        return dx

    @staticmethod
    def _k26_ok(conv, x0):
        return x0.dtype == torch.uint8 and conv.weight.grad.is_contiguous() and conv.bias.grad.is_contiguous()

    def _conv1_wgrad(self, conv, g, xu, act=None):
        """K26 partials + the f64 column-sum finalize -> conv.weight.grad.  act None: g is d output after the
        activation backward (K22 / K24 ran); act = (code, slope, y): g is d loss / d y and K26 also forms the
        activation backward and the bias-gradient partials (-> conv.bias.grad)."""
        L, st = ops.lib(), ops._stream(g.device)
        G = int(L.xpa_conv1_u8_wgrad_num_partials())
        if getattr(self, "_wg_part", None) is None:
            self._wg_part = torch.empty((G, 8192), dtype=torch.float32, device=g.device)
            self._wb_part = torch.empty((G, 32), dtype=torch.float32, device=g.device)
        g = g if g.is_contiguous() else g.contiguous()
        B, H, W, C = xu.shape
        code, slope, y = act if act is not None else (-1, 0.0, None)
        _lib.check(L.xpa_conv1_u8_wgrad_act(code, ops._p(g), ops._p(y) if y is not None else None, float(slope),
                                            ops._p(xu), B, H, W, C, 8, conv.stride[0], conv.padding[0], 32,
                                            ops._p(self._wg_part), ops._p(self._wb_part) if y is not None else None,
                                            st), "xpa_conv1_u8_wgrad_act")
        _lib.check(L.xpa_colsum_finalize(ops._p(self._wg_part), G, 8192, ops._p(conv.weight.grad), st),
                   "xpa_colsum_finalize")
        if y is not None:
            _lib.check(L.xpa_colsum_finalize(ops._p(self._wb_part), G, 32, ops._p(conv.bias.grad), st),
                       "xpa_colsum_finalize")

    @staticmethod
    def _dgrad_ok(conv):
        """K27 takes the data gradient of 2s x 2s, stride-s (1, 2) convs with 32 -> 64 channels."""
        k, st, pd = conv.kernel_size, conv.stride, conv.padding
        return (conv.in_channels == 32 and conv.out_channels == 64 and k[0] == k[1] and st[0] == st[1]
                and pd[0] == pd[1] and st[0] in (1, 2) and k[0] == 2 * st[0] and pd[0] < k[0]
                and conv.padding_mode == "zeros" and conv.weight.is_contiguous())

    @staticmethod
    def _dgrad(conv, g, in_shape):
        """K27: d input (NHWC [B, H, W, 32]) from g = d output (NHWC [B, OH, OW, 64], contiguous)."""
        B, H, W = in_shape[0], in_shape[1], in_shape[2]
        dx = torch.empty((B, H, W, 32), dtype=torch.float32, device=g.device)
        _lib.check(ops.lib().xpa_conv_dgrad_s2k(ops._p(g), B, g.shape[1], g.shape[2], 64, ops._p(conv.weight), 32,
                                                conv.kernel_size[0], conv.stride[0], conv.padding[0], H, W, ops._p(dx),
                                                ops._stream(g.device)), "xpa_conv_dgrad_s2k")
        return dx

    @torch.no_grad()
    def backward(self, ctx, ds):
        """ds: d loss / d state [B, d]; writes every trunk parameter's gradient."""
        hs, am, flat, fouts = ctx
        B = hs[0].shape[0]
        parts = self.parts
        g = ds
        fused_dz = False   # g leaves the fc part as the last conv block's dz (its K22 done in the fc epilogue)
        if self.tail == "flatten":
            for j in range(len(self.fc) - 1, -1, -1):
                lin, code, slope = self.fc[j]
                x_in = flat if j == 0 else fouts[j - 1]
                g = g.contiguous()
                _act_bwd_bias(parts, code, g, fouts[j], slope, lin.bias.grad)
                if j == 0:
                    if self._dw_tmp is None:
                        self._dw_tmp = torch.empty_like(lin.weight)
                    if not self._fc0_wgrad_split(g, x_in):
                        torch.mm(g.t(), x_in, out=self._dw_tmp)
                    Cl, Hl, Wl = self._chw
                    lin.weight.grad.view(lin.out_features, Cl, Hl, Wl).copy_(
                        self._dw_tmp.view(lin.out_features, Hl, Wl, Cl).permute(0, 3, 1, 2))
                    if self._fc_fuse_ok(g.shape[0]) and flat.is_contiguous():
                        g = self._fc0_dgrad_split_act(g, flat)
                        fused_dz = True
                    elif self._fc_split_ok(g.shape[0]):
                        g = self._fc0_dgrad_split(g)
                    else:
                        g = torch.mm(g, self._fc0_weight())
                else:
                    torch.mm(g.t(), x_in, out=lin.weight.grad)
                    g = torch.mm(g, lin.weight)
        # conv blocks, last to first.  g is the NHWC gradient of the block's output (after its activation), or — once
        # a fused step has applied the activation backward (K24 for the max-pool tail, K28's data gradient epilogue) —
        # its pre-activation gradient dz (g_dz), with that block's bias gradient already written.
        g_dz = fused_dz
        for i in range(len(self.convs) - 1, -1, -1):
            conv, code, slope = self.convs[i]
            y = hs[i + 1]
            Cy = y.shape[3]
            if i == len(self.convs) - 1 and self.tail == "maxpool":
                HW = y.shape[1] * y.shape[2]
                dz = torch.empty_like(y)
                part = parts.get(B * HW, Cy, y.device, True)
                L, st = ops.lib(), ops._stream(y.device)
                if getattr(self, "err", None) is None:
                    self.err = torch.zeros((1,), dtype=torch.int32, device=y.device)   # argmax outside [0, HW)
                _lib.check(L.xpa_maxpool_act_bwd_bias(code, ops._p(ds.contiguous()), ops._p(am), ops._p(y), B, HW, Cy,
                                                      float(slope), ops._p(dz), ops._p(part), ops._p(self.err), st),
                           "xpa_maxpool_act_bwd_bias")
                _lib.check(L.xpa_colsum_finalize(ops._p(part), part.shape[0], Cy, ops._p(conv.bias.grad), st),
                           "xpa_colsum_finalize")
                g, g_dz = dz, True
            else:
                g = g.reshape(y.shape)
                if not g.is_contiguous():
                    g = g.contiguous()
            if i == 0 and self._k26_ok(conv, hs[0]):
                # K26 from the uint8 frames: with the activation backward + bias gradient folded in unless done
                self._conv1_wgrad(conv, g, hs[0], act=None if g_dz else (code, slope, y))
                break
            x_in = self.frames(hs[i]) if hs[i].dtype == torch.uint8 else hs[i]
            numel = max(x_in.numel(), g.numel())
            rows = y.shape[0] * y.shape[1] * y.shape[2]
            ig = self._igemm_ok(conv, numel, rows)
            need_in = i > 0
            if not g_dz and (need_in or not ig):
                # the data gradient (and the library weight gradient) read dz: K22 in place, + the bias gradient
                _act_bwd_bias(parts, code, g.view(-1, Cy), y.view(-1, Cy), slope, conv.bias.grad)
                g_dz = True
            if ig:   # K29 (with the activation backward + bias gradient folded in when g is not dz yet)
                self._conv_wgrad(conv, g, -1 if g_dz else code, slope, y, x_in)
            if not ig or (need_in and not self._dgrad_ok(conv) and not self._igemm_dgrad_ok(conv, numel, rows)):
                k27 = need_in and self._dgrad_ok(conv)
                _library_conv_guard(conv)
                gx, gw, _ = torch.ops.aten.convolution_backward(
                    g.permute(0, 3, 1, 2), x_in.permute(0, 3, 1, 2), conv.weight, None, list(conv.stride),
                    list(conv.padding), [1, 1], False, [0, 0], 1, [need_in and not k27, not ig, False])
                if not ig:
                    conv.weight.grad.copy_(gw)
                if need_in and not k27:
                    g, g_dz = gx.permute(0, 2, 3, 1), False
                    continue
            if not need_in:
                break
            if self._dgrad_ok(conv):   # K27 (the stride-2 32 -> 64 conv): the previous block's g, not dz
                g, g_dz = self._dgrad(conv, g, x_in.shape), False
            else:                      # K28's data gradient with the previous block's activation backward + bias
                pconv, pcode, pslope = self.convs[i - 1]
                g = self._conv_dgrad(conv, g, tuple(x_in.shape), (pcode, pslope, hs[i], pconv.bias.grad))
                g_dz = True
        self.stale = True   # the optimizer step that follows changes the fc weight


class FusedCNNActorCritic:
    """Built from a Categorical/Gaussian actor-critic policy with an AC_CNN_Atari representation."""

    def __init__(self, policy):
        self.parts = _Part()
        self.trunk_ = _Trunk(policy.representation, self.parts)
        if self.trunk_.tail != "flatten":
            raise ValueError("the actor-critic path expects AC_CNN_Atari")
        self.discrete = policy_discrete(policy)
        self.actor = _parse(policy.actor.model if self.discrete else policy.actor.mu)
        self.critic = _parse(policy.critic.model)
        self.logstd = None if self.discrete else policy.actor.logstd
        n_params = sum(1 for _ in policy.parameters())
        n_cov = self.trunk_.n_params + 2 * (len(self.actor) + len(self.critic)) + (0 if self.discrete else 1)
        if n_params != n_cov:
            raise ValueError("policy has parameters outside the conv / Linear chains")

    @property
    def stale(self):
        return self.trunk_.stale

    @stale.setter
    def stale(self, v):
        self.trunk_.stale = v

    def refresh(self):
        """Re-derive the (H, W, C)-ordered first fc weight now (the agent calls it before a captured rollout, whose
        graph must not contain the copy)."""
        self.trunk_.refresh()

    def frames(self, x):
        return self.trunk_.frames(x)

    @torch.no_grad()
    def trunk(self, x):
        return self.trunk_.forward(x)

    @torch.no_grad()
    def forward(self, x):
        """(logits or mu, logstd or None, v, ctx)."""
        s, tctx = self.trunk_.forward(x)
        a_outs = _chain(self.actor, s)
        c_outs = _chain(self.critic, s)
        return a_outs[-1], self.logstd, c_outs[-1][:, 0], (tctx, s, a_outs, c_outs)

    @torch.no_grad()
    def heads(self, x):
        head, logstd, v, _ = self.forward(x)
        return head, logstd, v

    @torch.no_grad()
    def backward(self, ctx, d_head, d_v):
        """Writes every parameter gradient (d_head [B, K], d_v [B]: the loss kernel's outputs)."""
        tctx, s, a_outs, c_outs = ctx
        ds = _chain_backward(self.parts, self.actor, [s] + a_outs[:-1], a_outs, d_head)
        ds = _chain_backward(self.parts, self.critic, [s] + c_outs[:-1], c_outs, d_v.view(-1, 1), acc=ds)
        self.trunk_.backward(tctx, ds)


class FusedQNetwork:
    """BasicQnetwork over a Basic_CNN (or AC_CNN_Atari) representation: explicit eval forward / backward and the
    target forward (deterministic.py:148-182)."""

    def __init__(self, policy):
        self.parts = _Part()
        self.eval_trunk = _Trunk(policy.representation, self.parts)
        self.target_trunk = _Trunk(policy.target_representation, self.parts)
        self.eval_head = _parse(policy.eval_Qhead.model)
        self.target_head = _parse(policy.target_Qhead.model)
        n_params = sum(1 for _ in policy.parameters())
        n_cov = 2 * self.eval_trunk.n_params + 4 * len(self.eval_head)
        if n_params != n_cov:
            raise ValueError("Q-network has parameters outside the conv / Linear chains")
        self.eval_params = self.eval_trunk.params() + [t for lin, _, _ in self.eval_head for t in (lin.weight, lin.bias)]

    @torch.no_grad()
    def forward(self, x):
        """evalQ [B, A] and the backward context."""
        s, tctx = self.eval_trunk.forward(x)
        outs = _chain(self.eval_head, s)
        return outs[-1], (tctx, s, outs)

    @torch.no_grad()
    def target(self, x):
        if self.target_trunk.tail == "flatten":
            self.target_trunk.stale = True   # copy_target() may have changed it since the last call
        s, _ = self.target_trunk.forward(x)
        return _chain(self.target_head, s)[-1]

    @torch.no_grad()
    def backward(self, ctx, dq):
        """dq = d loss / d evalQ [B, A] (K19); writes every eval parameter's gradient."""
        _ensure_grads(self.eval_params)
        tctx, s, outs = ctx
        ds = _chain_backward(self.parts, self.eval_head, [s] + outs[:-1], outs, dq.contiguous())
        self.eval_trunk.backward(tctx, ds)

    def refresh(self):
        self.eval_trunk.refresh()
        self.target_trunk.refresh()
