"""Actor-critic networks and distributions with the reference's interface and state_dict layout.

Mirrors (reference paths):
  mlp_block / cnn_block          xuance/torch/utils/layers.py:8-57
  Basic_Identical / Basic_MLP    xuance/torch/representations/mlp.py:5-51
  AC_CNN_Atari                   xuance/torch/representations/cnn.py:45-93
  Gaussian_AC_Policy             xuance/torch/policies/gaussian.py:8-77
  Categorical_AC_Policy          xuance/torch/policies/categorical.py:16-85
  distributions                  xuance/torch/utils/distributions.py:39-101
State-dict keys match the reference's (representation.model.*, actor.mu.* / actor.model.*,
actor.logstd, critic.model.*), so checkpoints load in either direction.

The GEMMs stay in PyTorch-ROCm (hipBLASLt); the hot path calls `heads(x)` (mu/logits, logstd, v as
plain tensors) instead of building torch.distributions objects, and the loss/gradient of the heads is
computed by the fused HIP kernel (xuanpolicy_amd.learners).
"""
from typing import Callable, Optional, Sequence, Type

import numpy as np
import torch
import torch.nn as nn

ModuleType = Type[nn.Module]

ActivationFunctions = {
    "ReLU": nn.ReLU, "LeakyReLU": nn.LeakyReLU, "Tanh": nn.Tanh, "Sigmoid": nn.Sigmoid, "Softmax": nn.Softmax,
    "Elu": nn.ELU,
}
NormalizeFunctions = {"LayerNorm": nn.LayerNorm, "BatchNorm": nn.BatchNorm1d}
InitializeFunctions = {"orthogonal": torch.nn.init.orthogonal_}


def space_shape(space):
    """space2shape (xuance/common/common_tools.py:185-189) for Box/Discrete-like objects."""
    if hasattr(space, "n") and not getattr(space, "shape", None):
        return ()
    return tuple(space.shape)


def _splitk_splits(batch, n_out, n_in):
    """Split count for the weight-gradient GEMM dW = dY^T X with K = batch.  hipBLASLt runs these
    long-K, small-M*N shapes without split-K (~32 workgroups on a 256-CU chip: 39 TF/s at 256x256,
    <3 TF/s at 256x17, measured r01); a batched GEMM over S slices of K + a sum fills the chip
    (S chosen so S x tiles >= ~512 workgroups, 32x64 tiles)."""
    tiles = max(1, -(-n_out // 32)) * max(1, -(-n_in // 64))
    s = 1
    while s * tiles < 512 and s < 64:
        s *= 2
    while s > 1 and (batch % s or batch // s < 512):
        s //= 2
    return s


class _SplitKLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return torch.nn.functional.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = gy.mm(w)
        if ctx.needs_input_grad[1]:
            B, n_out, n_in = x.shape[0], w.shape[0], w.shape[1]
            s = _splitk_splits(B, n_out, n_in)
            if s > 1:
                gyc, xc = gy.contiguous(), x.contiguous()
                gw = torch.bmm(gyc.view(s, B // s, n_out).transpose(1, 2), xc.view(s, B // s, n_in)).sum(0)
            else:
                gw = gy.t().mm(x)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = gy.sum(0)
        return gx, gw, gb


class FastLinear(nn.Linear):
    """nn.Linear (same parameters and state_dict) whose backward computes the weight gradient of
    large batches as a split-K batched GEMM (see _splitk_splits)."""

    min_batch = 8192

    def forward(self, x):
        if x.dim() == 2 and x.shape[0] >= self.min_batch and torch.is_grad_enabled() and x.is_cuda:
            return _SplitKLinearFn.apply(x, self.weight, self.bias)
        return torch.nn.functional.linear(x, self.weight, self.bias)


def mlp_block(input_dim, output_dim, normalize=None, activation=None, initialize=None, device=None):
    """Linear -> activation -> normalize (layers.py:8-24)."""
    block = []
    linear = FastLinear(input_dim, output_dim, device=device)
    if initialize is not None:
        initialize(linear.weight)
        nn.init.constant_(linear.bias, 0)
    block.append(linear)
    if activation is not None:
        block.append(activation())
    if normalize is not None:
        block.append(normalize(output_dim, device=device))
    return block, (output_dim,)


def cnn_block(input_shape, filters, kernel_size, stride, normalize=None, activation=None, initialize=None,
              device=None):
    """Conv2d with padding (k - s) // 2 -> activation (layers.py:27-57)."""
    C, H, W = input_shape
    padding = int((kernel_size - stride) // 2)
    cnn = nn.Conv2d(C, filters, kernel_size, stride, padding=padding, device=device)
    if initialize is not None:
        initialize(cnn.weight)
        nn.init.constant_(cnn.bias, 0)
    block = [cnn]
    H = int((H + 2 * padding - (kernel_size - 1) - 1) / stride + 1)
    W = int((W + 2 * padding - (kernel_size - 1) - 1) / stride + 1)
    if activation is not None:
        block.append(activation())
    if normalize is not None:
        block.append(normalize(filters, device=device))
    return block, (filters, H, W)


def _as_input(observations, device, dtype=torch.float32):
    if isinstance(observations, torch.Tensor):
        t = observations
        if device is not None and t.device != torch.device(device):
            t = t.to(device)
        return t if t.dtype == dtype else t.to(dtype)
    return torch.as_tensor(np.asarray(observations), dtype=dtype, device=device)


class Basic_Identical(nn.Module):
    def __init__(self, input_shape: Sequence[int], device=None):
        super().__init__()
        assert len(input_shape) == 1
        self.output_shapes = {"state": (input_shape[0],)}
        self.device = device
        self.model = nn.Sequential()

    def forward(self, observations):
        return {"state": _as_input(observations, self.device)}


class Basic_MLP(nn.Module):
    def __init__(self, input_shape: Sequence[int], hidden_sizes: Sequence[int], normalize: Optional[ModuleType] = None,
                 initialize: Optional[Callable] = None, activation: Optional[ModuleType] = None, device=None):
        super().__init__()
        self.input_shape, self.hidden_sizes = tuple(input_shape), list(hidden_sizes)
        self.device = device
        self.output_shapes = {"state": (self.hidden_sizes[-1],)}
        layers, shape = [], self.input_shape
        for h in self.hidden_sizes:
            mlp, shape = mlp_block(shape[0], h, normalize, activation, initialize, device)
            layers.extend(mlp)
        self.model = nn.Sequential(*layers)

    def forward(self, observations):
        return {"state": self.model(_as_input(observations, self.device))}


class AC_CNN_Atari(nn.Module):
    """cnn.py:45-93.  Input uint8 [B, 84, 84, C] (NHWC); /255 and NHWC->NCHW happen on device here
    (the reference does them on the host per minibatch, cnn.py:89-92)."""

    def __init__(self, input_shape, kernels, strides, filters, normalize=None, initialize=None, activation=None,
                 device=None, fc_hidden_sizes=()):
        super().__init__()
        self.input_shape = (input_shape[2], input_shape[0], input_shape[1])
        self.device = device
        self.output_shapes = {"state": (fc_hidden_sizes[-1],)}
        layers, shape = [], self.input_shape
        for k, s, f in zip(kernels, strides, filters):
            cnn, shape = cnn_block(shape, f, k, s, None, activation, None, device)
            nn.init.orthogonal_(cnn[0].weight, gain=np.sqrt(2))
            nn.init.constant_(cnn[0].bias, 0)
            layers.extend(cnn)
        layers.append(nn.Flatten())
        shape = (int(np.prod(shape)),)
        for h in fc_hidden_sizes:
            mlp, shape = mlp_block(shape[0], h, None, activation, None, device)
            nn.init.orthogonal_(mlp[0].weight, gain=np.sqrt(2))
            nn.init.constant_(mlp[0].bias, 0)
            layers.extend(mlp)
        self.model = nn.Sequential(*layers)

    def forward(self, observations):
        x = _as_input(observations, self.device, dtype=torch.float32) / 255.0
        return {"state": self.model(x.permute(0, 3, 1, 2))}


class Basic_CNN(nn.Module):
    """cnn.py:5-40: conv blocks (padding (k - s) // 2, activation) + global max pool + flatten; state dim =
    filters[-1].  Input uint8 [B, 84, 84, C] (NHWC): /255 and the NCHW view happen on device."""

    def __init__(self, input_shape, kernels, strides, filters, normalize=None, initialize=None, activation=None,
                 device=None):
        super().__init__()
        self.input_shape = (input_shape[2], input_shape[0], input_shape[1])
        self.device = device
        self.output_shapes = {"state": (filters[-1],)}
        layers, shape = [], self.input_shape
        for k, s, f in zip(kernels, strides, filters):
            cnn, shape = cnn_block(shape, f, k, s, normalize, activation, initialize, device)
            layers.extend(cnn)
        layers.append(nn.AdaptiveMaxPool2d((1, 1)))
        layers.append(nn.Flatten())
        self.model = nn.Sequential(*layers)

    def forward(self, observations):
        x = _as_input(observations, self.device, dtype=torch.float32) / 255.0
        return {"state": self.model(x.permute(0, 3, 1, 2))}


class BasicQhead(nn.Module):
    """deterministic.py:6-25."""

    def __init__(self, state_dim, action_dim, hidden_sizes, normalize=None, initialize=None, activation=None,
                 device=None):
        super().__init__()
        layers, shape = [], (state_dim,)
        for h in hidden_sizes:
            mlp, shape = mlp_block(shape[0], h, normalize, activation, initialize, device)
            layers.extend(mlp)
        layers.extend(mlp_block(shape[0], action_dim, None, None, None, device)[0])
        self.model = nn.Sequential(*layers)

    def forward(self, x):
        return self.model(x)


class BasicQnetwork(nn.Module):
    """deterministic.py:148-182 (the same module names, so the reference's checkpoints load): an evaluation
    network, a target network (deep copies), copy_target() for the hard update."""

    def __init__(self, action_space, representation, hidden_size=None, normalize=None, initialize=None,
                 activation=None, device=None):
        super().__init__()
        import copy
        self.action_dim = action_space.n
        self.representation = representation
        self.target_representation = copy.deepcopy(representation)
        self.representation_info_shape = self.representation.output_shapes
        self.eval_Qhead = BasicQhead(self.representation.output_shapes["state"][0], self.action_dim,
                                     hidden_size or [], normalize, initialize, activation, device)
        self.target_Qhead = copy.deepcopy(self.eval_Qhead)

    def forward(self, observation):
        outputs = self.representation(observation)
        evalQ = self.eval_Qhead(outputs["state"])
        return outputs, evalQ.argmax(dim=-1), evalQ

    def target(self, observation):
        outputs = self.target_representation(observation)
        targetQ = self.target_Qhead(outputs["state"])
        return outputs, targetQ.argmax(dim=-1).detach(), targetQ.detach()

    def copy_target(self):
        with torch.no_grad():
            for ep, tp in zip(self.representation.parameters(), self.target_representation.parameters()):
                tp.copy_(ep)
            for ep, tp in zip(self.eval_Qhead.parameters(), self.target_Qhead.parameters()):
                tp.copy_(ep)


class CategoricalDistribution:
    """distributions.py:39-66."""

    def __init__(self, action_dim):
        self.action_dim = action_dim

    def set_param(self, logits):
        self.logits = logits
        self.distribution = torch.distributions.Categorical(logits=logits)

    def get_param(self):
        return self.logits

    def log_prob(self, x):
        return self.distribution.log_prob(x)

    def entropy(self):
        return self.distribution.entropy()

    def stochastic_sample(self):
        return self.distribution.sample()

    def deterministic_sample(self):
        return torch.argmax(self.distribution.probs, dim=1)


class DiagGaussianDistribution:
    """distributions.py:69-101."""

    def __init__(self, action_dim):
        self.action_dim = action_dim
        self.mu = self.std = None

    def set_param(self, mu, std):
        self.mu, self.std = mu, std
        self.distribution = torch.distributions.Normal(mu, std)

    def get_param(self):
        return self.mu, self.std

    def log_prob(self, x):
        return self.distribution.log_prob(x).sum(-1)

    def entropy(self):
        return self.distribution.entropy().sum(-1)

    def stochastic_sample(self):
        return self.distribution.sample()

    def deterministic_sample(self):
        return self.mu


class _GaussianActor(nn.Module):
    def __init__(self, state_dim, action_dim, hidden_sizes, normalize, initialize, activation, device):
        super().__init__()
        layers, shape = [], (state_dim,)
        for h in hidden_sizes:
            mlp, shape = mlp_block(shape[0], h, normalize, activation, initialize, device)
            layers.extend(mlp)
        layers.extend(mlp_block(shape[0], action_dim, None, None, initialize, device)[0])
        self.mu = nn.Sequential(*layers)
        self.logstd = nn.Parameter(-torch.ones((action_dim,), device=device))
        self.dist = DiagGaussianDistribution(action_dim)

    def forward(self, x):
        self.dist.set_param(self.mu(x), self.logstd.exp())
        return self.dist


class _CategoricalActor(nn.Module):
    def __init__(self, state_dim, action_dim, hidden_sizes, normalize, initialize, activation, device):
        super().__init__()
        layers, shape = [], (state_dim,)
        for h in hidden_sizes:
            mlp, shape = mlp_block(shape[0], h, normalize, activation, initialize, device)
            layers.extend(mlp)
        layers.extend(mlp_block(shape[0], action_dim, None, None, initialize, device)[0])
        self.model = nn.Sequential(*layers)
        self.dist = CategoricalDistribution(action_dim)

    def forward(self, x):
        self.dist.set_param(self.model(x))
        return self.dist


class _Critic(nn.Module):
    def __init__(self, state_dim, hidden_sizes, normalize, initialize, activation, device, init_last):
        super().__init__()
        layers, shape = [], (state_dim,)
        for h in hidden_sizes:
            mlp, shape = mlp_block(shape[0], h, normalize, activation, initialize, device)
            layers.extend(mlp)
        layers.extend(mlp_block(shape[0], 1, None, None, initialize if init_last else None, device)[0])
        self.model = nn.Sequential(*layers)

    def forward(self, x):
        return self.model(x)[:, 0]


class _ActorCritic(nn.Module):
    discrete = False

    def forward(self, observation):
        outputs = self.representation(observation)
        a = self.actor(outputs["state"])
        v = self.critic(outputs["state"])
        return outputs, a, v

    # ---- fused hot path -------------------------------------------------------------------------
    def heads(self, x):
        """(mu or logits, logstd or None, v) for a float32 device tensor x — no distribution objects."""
        s = self.representation(x)["state"]
        if self.discrete:
            return self.actor.model(s), None, self.critic(s)
        return self.actor.mu(s), self.actor.logstd, self.critic(s)

    def value(self, x):
        return self.critic(self.representation(x)["state"])


class Gaussian_AC_Policy(_ActorCritic):
    """gaussian.py:54-77 (the critic's last layer keeps torch's default init, gaussian.py:47)."""

    def __init__(self, action_space, representation, actor_hidden_size=None, critic_hidden_size=None, normalize=None,
                 initialize=None, activation=None, device=None):
        super().__init__()
        self.action_dim = action_space.shape[0]
        self.representation = representation
        self.representation_info_shape = representation.output_shapes
        d = representation.output_shapes["state"][0]
        self.actor = _GaussianActor(d, self.action_dim, actor_hidden_size or [], normalize, initialize, activation,
                                    device)
        self.critic = _Critic(d, critic_hidden_size or [], normalize, initialize, activation, device, init_last=False)


class Categorical_AC_Policy(_ActorCritic):
    """categorical.py:61-85."""
    discrete = True

    def __init__(self, action_space, representation, actor_hidden_size=None, critic_hidden_size=None, normalize=None,
                 initialize=None, activation=None, device=None):
        super().__init__()
        self.device = device
        self.action_dim = action_space.n
        self.representation = representation
        self.representation_info_shape = representation.output_shapes
        d = representation.output_shapes["state"][0]
        self.actor = _CategoricalActor(d, self.action_dim, actor_hidden_size or [], normalize, initialize, activation,
                                       device)
        self.critic = _Critic(d, critic_hidden_size or [], normalize, initialize, activation, device, init_last=True)


REGISTRY = {"Gaussian_AC": Gaussian_AC_Policy, "Categorical_AC": Categorical_AC_Policy, "Basic_Q_network": BasicQnetwork}
REGISTRY_Representation = {"Basic_Identical": Basic_Identical, "Basic_MLP": Basic_MLP, "AC_CNN_Atari": AC_CNN_Atari,
                           "Basic_CNN": Basic_CNN}


def policy_discrete(policy):
    """Categorical when the actor has no logstd: categorical.py's ActorNet holds .model, gaussian.py's .mu + .logstd
    (the reference's classes carry no `discrete` attribute; ours do, with the same meaning)."""
    d = getattr(policy, "discrete", None)
    return bool(d) if d is not None else not hasattr(policy.actor, "logstd")


def policy_heads(policy, x):
    """(head, logstd, v) for our policies or the reference's classes (same attribute layout)."""
    if hasattr(policy, "heads"):
        return policy.heads(x)
    s = policy.representation(x)["state"]
    if hasattr(policy.actor, "logstd"):
        return policy.actor.mu(s), policy.actor.logstd, policy.critic(s)
    return policy.actor.model(s), None, policy.critic(s)
