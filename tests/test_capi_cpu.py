"""CPU tests of the drop-in boundary: the C-ABI library builds, loads and exports every symbol that
include/xuanpolicy_amd.h declares; the Python bindings cover them; no compute call without a GPU."""
import os
import re
import subprocess

import pytest
import torch

from xuanpolicy_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    src = open(os.path.join(REPO, "include", "xuanpolicy_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(xpa_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    _lib.build_library()
    return _lib.load()


def test_header_symbols_exported(lib):
    names = _header_functions()
    assert len(names) >= 15
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (xpa_\w+)", out))
    assert set(names) == exported, (set(names) ^ exported)
    for n in names:
        assert hasattr(lib, n)


def test_bindings_cover_header():
    assert set(_header_functions()) == set(_lib.SIGNATURES)


def test_abi_version_and_size_helpers(lib):
    assert lib.xpa_abi_version() == _lib.ABI_VERSION
    assert lib.xpa_loss_num_partials(65536) == 256 and lib.xpa_loss_num_partials(1 << 22) == 2048
    assert lib.xpa_loss_partial_width(6) == 11
    assert lib.xpa_gather_num_partials(65537) == 1025
    assert lib.xpa_rms_num_partials(4096) == 16


def test_invalid_arguments_rejected_before_launch(lib):
    # null pointers / bad shapes return hipErrorInvalidValue (1) without touching a device
    assert lib.xpa_gae_scan(None, None, None, None, None, 4, 4, 0.99, 0.95, 1, None, None, None) == 1
    assert lib.xpa_gae_scan(None, None, None, None, None, -1, 4, 0.99, 0.95, 1, None, None, None) == 1
    assert lib.xpa_policy_loss_fwd_bwd(0, 0, 0, 6, *([None] * 4), 1, *([None] * 5), 0, 0.2, 0.25, 0.0,
                                       None, None, None, None) == 1
    assert lib.xpa_policy_loss_fwd_bwd(0, 1, 8, 1, *([None] * 4), 8, *([None] * 5), 0, 0.2, 0.25, 0.0,
                                       None, None, None, None) == 1
    assert lib.xpa_gather_minibatch(None, 8, 8, None, 4, None, None, None, None, None) == 1
    assert lib.xpa_rms_merge(None, 3, 100, 4, None, None, None, None) == 1
    # K16X: the trunk width (d_in <= 20), the head width (<= 8) and h_out's alignment are checked before any launch
    # (fake, 16-B aligned non-null pointers elsewhere, so only the checked argument can fail)
    import ctypes
    P = ctypes.c_void_p(256)

    def trunk_actor(act_dim=6, d_in=17, h_out=P):
        return lib.xpa_head_gemm_trunk_actor(0, 0, 1, 64, act_dim, 256, P, d_in, d_in, P, P, 0.01, h_out, 256, P, P,
                                             512, P, P, 0.01, P, P, 100, P, P, P, P, 1, 0.2, 0.0, P, P, P, P, P, 16, None)
    assert trunk_actor(d_in=21) == 1
    assert trunk_actor(act_dim=9) == 1
    assert trunk_actor(h_out=ctypes.c_void_p(260)) == 1
    assert lib.xpa_head_gemm_trunk_critic(1, 64, 256, P, 21, 21, P, P, 0.01, None, 256, P, P, 512, P, P, 0.01, P, 100,
                                          P, 0.25, P, P, P, P, P, 16, None) == 1
    # the gather-only K13 form needs the rows output when h is NULL
    assert lib.xpa_thin_linear_act_fwd_gather(1, P, 17, 100, P, 64, 17, 256, P, P, 0.01, None, 256, P, P, None,
                                              None) == 1


def test_ops_refuse_cpu_tensors():
    from xuanpolicy_amd import ops
    x = torch.zeros(4, 8)
    with pytest.raises(ValueError, match="ROCm device"):
        ops.gae_scan(x, x, x, torch.zeros(4, 8, dtype=torch.uint8), x, 0.99, 0.95)
    with pytest.raises(ValueError, match="ROCm device"):
        ops.policy_loss("ppo", "gaussian", torch.zeros(4, 2), torch.zeros(2), torch.zeros(4), torch.zeros(8),
                        torch.zeros(4), torch.zeros(4), old_logp=torch.zeros(4))


def test_config_cascade():
    from xuanpolicy_amd.runner import get_arguments
    a = get_arguments("ppo", "synthbox", "SynthBox-v0")
    assert (a.agent, a.parallels, a.n_steps, a.n_epoch, a.n_minibatch) == ("PPO_Clip", 4096, 128, 16, 8)
    assert a.representation_hidden_size == [256] and a.clip_grad_norm == 0.5 and a.use_obsnorm
    b = get_arguments("a2c", "synthbox", "SynthBox-v0")
    assert b.agent == "A2C" and b.discrete and b.clip_grad == 0.5


def test_registries_match_reference_names():
    from xuanpolicy_amd import agents, learners, policies
    assert set(agents.REGISTRY) == {"PPO_Clip", "A2C", "PerDQN"}
    assert set(learners.REGISTRY) == {"PPO_Clip", "A2C", "PerDQN"}
    assert {"Gaussian_AC", "Categorical_AC", "Basic_Q_network"} <= set(policies.REGISTRY)
    assert {"Basic_MLP", "AC_CNN_Atari", "Basic_CNN"} <= set(policies.REGISTRY_Representation)


def test_qnetwork_state_dict_keys_match_reference(golden):
    """BasicQnetwork over Basic_CNN loads the reference's state_dict (deterministic.py:148-182, cnn.py:5-40)."""
    import torch
    from xuanpolicy_amd.policies import BasicQnetwork, Basic_CNN
    g = golden("perdqn.npz")
    B, A = (int(x) for x in g["config"][:2])
    net = [int(x) for x in g["net"]]
    nl = (len(net) - 1) // 3

    class Disc:
        n, shape = A, ()
    rep = Basic_CNN((84, 84, 4), net[nl:2 * nl], net[2 * nl:3 * nl], net[:nl], None, None, torch.nn.ReLU, "cpu")
    pol = BasicQnetwork(Disc(), rep, net[3 * nl:], None, None, torch.nn.ReLU, "cpu")
    sd = {k[4:]: torch.as_tensor(v) for k, v in g.items() if k.startswith("sd0/")}
    assert set(pol.state_dict()) == set(sd)
    pol.load_state_dict(sd)


def test_policy_state_dict_keys_match_reference(golden):
    """Our Gaussian/Categorical AC modules load the reference's state_dict (checkpoint interchange)."""
    from xuanpolicy_amd.policies import Basic_MLP, Categorical_AC_Policy, Gaussian_AC_Policy

    class Box:
        shape = (6,)

    class Disc:
        n, shape = 6, ()
    g = golden("loss.npz")
    for tag, cls, space in (("ppo_gaussian_6", Gaussian_AC_Policy, Box()),
                            ("ppo_categorical_6", Categorical_AC_Policy, Disc())):
        D = g[tag + "/obs"].shape[1]
        rep = Basic_MLP((D,), [64], None, torch.nn.init.orthogonal_, torch.nn.LeakyReLU, "cpu")
        pol = cls(space, rep, [64], [64], None, torch.nn.init.orthogonal_, torch.nn.LeakyReLU, "cpu")
        sd = {k[len(tag) + 5:]: torch.as_tensor(v) for k, v in g.items() if k.startswith(tag + "/sd0/")}
        pol.load_state_dict(sd)
        out, dist, v = pol(g[tag + "/obs"])
        head = dist.mu if hasattr(dist, "mu") else dist.logits
        assert torch.allclose(head, torch.as_tensor(g[tag + "/head"]), atol=1e-5)
        assert torch.allclose(v, torch.as_tensor(g[tag + "/v"]), atol=1e-5)


def test_flat_state_placement_groups():
    """FlatState keeps parameter order/offsets per parameter but lays placement groups back to back
    (the paired actor|critic hidden layer of fused_mlp.head_placement)."""
    from xuanpolicy_amd.flat import ALIGN, FlatState
    from xuanpolicy_amd.fused_mlp import head_placement
    from xuanpolicy_amd.policies import Basic_MLP, Gaussian_AC_Policy

    class Box:
        shape = (6,)
    torch.manual_seed(0)
    rep = Basic_MLP((17,), [256], None, torch.nn.init.orthogonal_, torch.nn.LeakyReLU, "cpu")
    pol = Gaussian_AC_Policy(Box(), rep, [256], [256], None, torch.nn.init.orthogonal_, torch.nn.LeakyReLU, "cpu")
    before = {k: v.clone() for k, v in pol.state_dict().items()}
    groups = head_placement(pol)
    assert len(groups) == 2
    fs = FlatState(pol.parameters(), placement=groups)
    assert [id(p) for p in fs.params] == [id(p) for p in pol.parameters()]
    assert all(o % ALIGN == 0 for o in fs.offsets)
    for g in groups:
        pv, gv = fs.span(g)
        assert pv.numel() == sum(p.numel() for p in g)
        assert pv.data_ptr() == g[0].data_ptr() and gv.data_ptr() == g[0].grad.data_ptr()
    assert fs.span([groups[0][1], groups[0][0]]) is None   # wrong order is not back to back
    for k, v in pol.state_dict().items():
        assert torch.equal(v, before[k]), k
    # offsets are unique and do not overlap
    spans = sorted((o, o + p.numel()) for p, o in zip(fs.params, fs.offsets))
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
