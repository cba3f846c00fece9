"""GPU: rollout-side equivalences — deferred truncation bootstraps (one critic pass per iteration)
reproduce the per-step bootstrap of the reference's agent (ppoclip_agent.py:69-101)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("agent_name,max_ep", [("PPO_Clip", 100), ("A2C", 100), ("PPO_Clip", 20)])
def test_deferred_bootstrap_matches_per_step(agent_name, max_ep):
    """max_ep 20 < n_steps 64: up to 4 truncations per env and rollout, each in its own deferred slot."""
    from xuanpolicy_amd.runner import build_synthbox_ppo
    kw = dict(n_envs=512, n_steps=64, n_epoch=2, n_minibatch=4, device=DEV, agent=agent_name, max_episode_steps=max_ep)
    a = build_synthbox_ppo(defer_bootstrap=True, **kw)
    b = build_synthbox_ppo(defer_bootstrap=False, **kw)
    b.policy.load_state_dict(a.policy.state_dict())
    assert a.defer_boot and not b.defer_boot and a.n_slots == (1 if max_ep >= 64 else 4)
    for _ in range(3):   # 3 iterations: truncations (every 100 steps) fall mid-buffer
        for ag in (a, b):
            for _ in range(ag.n_steps - 1):
                ag.train(1)
        ma, mb = a.memory, b.memory
        # before the last step: closures identical; deferred bootstraps not yet written
        for ag in (a, b):
            ag.train(1)      # last step + update phase
        assert torch.equal(ma.closed, mb.closed)
        assert int(ma.closed[:, :-1].sum()) > 0
        torch.testing.assert_close(ma.boot, mb.boot, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(ma.advantages, mb.advantages, rtol=1e-4, atol=1e-4)
        assert int(a.slot_t.max()) == -1 and int(a.slot_overflow) == 0
    ia, ib = a.infos[0], b.infos[0]
    for k in ("actor-loss", "critic-loss", "entropy"):
        assert np.isclose(ia[k], ib[k], rtol=1e-3, atol=1e-5), (k, ia[k], ib[k])
