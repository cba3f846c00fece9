"""CPU: the lockstep replay's kink candidates (oracle/cpu_ref.py LearnerRef._kink_rows, r06).  A (row, unit) whose
pre-activation sits within the f32 GEMM's rounding of the LeakyReLU kink is found, and its candidate gradient is the
change of taking the kink's other side: (s_other - s) dL/dh(row, unit) grad_theta z(row, unit) — for a unit of the
first layer, nonzero only in that unit's weight row and bias, equal to (s_other - s) dL/dh x_row there."""
import numpy as np
import torch

from oracle import cpu_ref


def test_kink_candidate_is_the_other_side_gradient():
    torch.manual_seed(0)
    pol = cpu_ref.build_actor_critic_ref(5, 2, [8], [8], [8])
    B = 16
    obs = np.random.default_rng(1).normal(size=(B, 5)).astype(np.float32)
    lin0 = pol.representation.model[0]
    with torch.no_grad():   # row 3, unit 2 of the first layer: pre-activation ~1e-9 (inside the rounding window)
        z = float((torch.as_tensor(obs[3]) @ lin0.weight[2]).item())
        lin0.bias[2] = -z + 1e-9
    opt = torch.optim.Adam(pol.parameters(), lr=1e-4)
    lrn = cpu_ref.LearnerRef(pol, opt, None, "ppo", 0.25, 0.0, 0.2, 0.5, True)
    act = np.random.default_rng(2).normal(size=(B, 2)).astype(np.float32)
    ret = np.random.default_rng(3).normal(size=B).astype(np.float32)
    adv = np.random.default_rng(4).normal(size=B).astype(np.float32)
    old_logp = np.full(B, -2.5, dtype=np.float32)
    x = torch.as_tensor(obs)
    lrn.update(obs, act, ret, adv, old_logp, capture_grads=True)
    cands = lrn.boundary_grads
    assert len(cands) >= 1
    names = [n for n, _ in pol.named_parameters()]
    first = dict(zip(names, cands[0]))
    w0, b0 = first["representation.model.0.weight"], first["representation.model.0.bias"]
    # nonzero only in unit 2's row / bias of the first layer; nothing downstream
    assert float(w0[2].abs().sum()) > 0 and float(b0[2].abs()) > 0
    assert float(w0[[0, 1, 3, 4, 5, 6, 7]].abs().sum()) == 0 and float(b0[[0, 1, 3, 4, 5, 6, 7]].abs().sum()) == 0
    for n, g in first.items():
        if not n.startswith("representation.model.0."):
            assert float(g.abs().sum()) == 0, n
    # the weight row is the bias entry times x_row (grad_theta z = (x_row, 1))
    torch.testing.assert_close(w0[2], b0[2] * x[3], rtol=1e-5, atol=1e-9)
