"""Host-side argument checks of the drop-in learners (no GPU): categorical actions outside [0, n) raise, as
torch's Categorical.log_prob does in the reference learners (ppoclip_learner.py:32-35, a2c_learner.py:27-30),
before anything is uploaded."""
import numpy as np
import pytest
import torch


class _Disc:
    def __init__(self, n):
        self.n, self.shape = n, ()


def _learner(algo, A=4, D=5):
    from xuanpolicy_amd.learners import A2C_Learner, PPOCLIP_Learner
    from xuanpolicy_amd.policies import Basic_MLP, Categorical_AC_Policy
    rep = Basic_MLP((D,), [8], None, torch.nn.init.orthogonal_, torch.nn.ReLU, "cpu")
    pol = Categorical_AC_Policy(_Disc(A), rep, [8], [8], None, torch.nn.init.orthogonal_, torch.nn.ReLU, "cpu")
    opt = torch.optim.Adam(pol.parameters(), 1e-3)
    if algo == "ppo":
        return PPOCLIP_Learner(pol, opt, None, "cpu", "./", clip_grad_norm=0.5)
    return A2C_Learner(pol, opt, None, "cpu", "./", 0.25, 0.01, 0.5)


@pytest.mark.parametrize("algo", ["ppo", "a2c"])
@pytest.mark.parametrize("bad", [[0, 4, 1], [-1, 0, 2], [0.5, 1, 2], [np.nan, 1, 2]])
def test_categorical_actions_out_of_range_raise(algo, bad):
    lrn = _learner(algo)
    B = len(bad)
    obs, act, z = np.zeros((B, 5), np.float32), np.asarray(bad, np.float32), np.zeros(B, np.float32)
    with pytest.raises(ValueError, match="categorical actions"):
        if algo == "ppo":
            lrn.update(obs, act, z, z, z, z)
        else:
            lrn.update(obs, act, z, z)


def test_categorical_actions_in_range_pass_the_check():
    lrn = _learner("ppo")
    lrn._check_actions(np.array([0, 3, 2, 1], np.int64))
    lrn._check_actions(torch.tensor([0.0, 3.0]))
    lrn._check_actions(np.zeros((0,), np.float32))
