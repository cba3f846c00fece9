"""CPU: the import-swap surface of INTEGRATION.md.  Every name the reference's on-policy examples import
from `xuance` (examples/ppo/ppo_mujoco.py, ppo_atari.py; read as text when /root/reference is mounted)
resolves under `xuanpolicy_amd`, and the agent / runner methods those examples call exist with the
reference's signatures (agent.py:74-79, ppoclip_agent.py:59,113, runner_drl.py:77,100)."""
import ast
import inspect
import os
from argparse import Namespace

import pytest

REF_EXAMPLES = [os.path.join("/root/reference/examples/ppo", f) for f in ("ppo_mujoco.py", "ppo_atari.py")]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _imports(path):
    tree = ast.parse(open(path).read())
    for node in ast.walk(tree):
        if isinstance(node, ast.ImportFrom) and node.module and node.module.split(".")[0] == "xuance":
            yield node.module, [a.name for a in node.names]


@pytest.mark.parametrize("path", REF_EXAMPLES)
def test_reference_example_imports_resolve(path):
    if not os.path.exists(path):
        pytest.skip("reference not mounted")
    import importlib
    seen = 0
    for module, names in _imports(path):
        mod = importlib.import_module("xuanpolicy_amd" + module[len("xuance"):])
        for n in names:
            assert hasattr(mod, n), "%s.%s missing" % (mod.__name__, n)
            seen += 1
    assert seen >= 8


def test_agent_and_runner_methods_match_reference_calls():
    from xuanpolicy_amd.torch.agents import A2C_Agent, PPOCLIP_Agent, get_total_iters
    from xuanpolicy_amd.torch.runners import Runner_DRL
    for cls in (PPOCLIP_Agent, A2C_Agent):
        assert list(inspect.signature(cls.__init__).parameters)[1:7] == ["config", "envs", "policy", "optimizer",
                                                                         "scheduler", "device"]
        assert list(inspect.signature(cls.save_model).parameters)[1:] == ["model_name"]
        assert list(inspect.signature(cls.load_model).parameters)[1:] == ["path", "seed"]
        assert list(inspect.signature(cls.test).parameters)[1:] == ["env_fn", "test_episode"]
        assert list(inspect.signature(cls.train).parameters)[1:2] == ["train_steps"]
        assert callable(cls.finish) and callable(cls.log_infos)
    assert get_total_iters("PPO_Clip", Namespace(running_steps=123)) == 123
    assert callable(Runner_DRL.run) and callable(Runner_DRL.benchmark)


def test_config_cascade_matches_reference_rules():
    """common_tools.py:32-83: basic.yaml -> method yaml (<env>.yaml for the flat env families) -> the user
    yaml (relative to the working directory) -> parser args (override by name)."""
    from xuanpolicy_amd import get_arguments
    cwd = os.getcwd()
    os.chdir(REPO)
    try:
        parser = Namespace(method="ppo", env="synthbox", env_id="SynthBox-v0", test=0, device="cuda:3", benchmark=1,
                           config="examples/ppo_synthbox_config.yaml")
        args = get_arguments(parser.method, parser.env, parser.env_id, parser.config, parser)
    finally:
        os.chdir(cwd)
    assert args.env_id == "SynthBox-v0" and args.agent == "PPO_Clip" and args.env_name == "SynthBox"
    assert args.device == "cuda:3"                 # parser args win
    assert args.seed == 79811 and args.parallels == 4096 and args.n_steps == 128   # the user yaml wins over ppo/synthbox.yaml
    assert args.test_episode == 16 and args.dl_toolbox == "torch"
    # a non-flat env without a method config: basic.yaml only, env_id kept from the user's values
    args2 = get_arguments("ppo", "classic_control", "CartPole-v1")
    assert args2.env_id == "CartPole-v1" and args2.dl_toolbox == "torch"


def test_jsonl_logger(tmp_path):
    from xuanpolicy_amd.agents import _make_writer
    w = _make_writer("wandb", str(tmp_path / "log"))   # neither wandb nor tensorboard here: JSON lines
    w.write({"a": 1.5, "Episode-Steps": {"env-0": 3}}, 7)
    w.close()
    import json
    rec = json.loads(open(tmp_path / "log" / "scalars.jsonl").read().strip())
    assert rec == {"step": 7, "a": 1.5, "Episode-Steps/env-0": 3.0}
    assert _make_writer("none", str(tmp_path)) is None


def _layer_sig(layers):
    return [(lin.in_features, lin.out_features, code, slope) for lin, code, slope in layers]


@pytest.mark.parametrize("discrete", [False, True])
def test_reference_policy_objects_take_the_fast_path_plan(discrete):
    """examples/ppo/ppo_mujoco.py:43-58 builds the policy from the REFERENCE's classes (xuance.torch.representations
    .Basic_MLP + xuance.torch.policies.Gaussian_AC_Policy / Categorical_AC_Policy, which carry no `discrete`
    attribute).  The fast-path planner recognises networks by structure, so those objects get the same layer parse,
    the same fused-head / K13 / paired-hidden-layer plan and the same flat-buffer placement as the mirror classes —
    the device agent's fused update, not the generic fallback.  Imports the reference in this container only."""
    if not os.path.isdir("/root/reference"):
        pytest.skip("reference not mounted")
    import torch
    from tests.golden.ref_loader import import_reference
    import_reference()
    import gym
    from xuance.torch.policies import Categorical_AC_Policy as RefCat, Gaussian_AC_Policy as RefGauss
    from xuance.torch.representations import Basic_MLP as RefMLP
    from xuance.torch.utils import ActivationFunctions as RefAct
    from xuanpolicy_amd.fused_mlp import FusedActorCritic, head_placement
    from xuanpolicy_amd.policies import (ActivationFunctions, Basic_MLP, Categorical_AC_Policy, Gaussian_AC_Policy,
                                         policy_discrete)
    space = gym.spaces.Discrete(4) if discrete else gym.spaces.Box(-1, 1, (6,))
    init = torch.nn.init.orthogonal_

    def build(mlp, pol_cls, acts):
        rep = mlp(input_shape=(17,), hidden_sizes=[256], normalize=None, initialize=init, activation=acts["LeakyReLU"],
                  device="cpu")
        return pol_cls(action_space=space, representation=rep, actor_hidden_size=[256], critic_hidden_size=[256],
                       normalize=None, initialize=init, activation=acts["LeakyReLU"], device="cpu")
    ref = build(RefMLP, RefCat if discrete else RefGauss, RefAct)
    ours = build(Basic_MLP, Categorical_AC_Policy if discrete else Gaussian_AC_Policy, ActivationFunctions)
    assert not hasattr(ref, "discrete") and policy_discrete(ref) == policy_discrete(ours) == discrete
    assert list(ref.state_dict().keys()) == list(ours.state_dict().keys())
    fr, fo = FusedActorCritic(ref), FusedActorCritic(ours)
    for part in ("rep", "actor", "critic"):
        assert _layer_sig(getattr(fr, part)) == _layer_sig(getattr(fo, part)), part
    for flag in ("discrete", "fused_heads", "thin0", "trunk_heads"):
        assert getattr(fr, flag) == getattr(fo, flag), flag
    assert fr.fused_heads and fr.thin0   # the C2 plan: K13 trunk + fused heads (K16 once the flat buffers pair them)
    hr, ho = head_placement(ref), head_placement(ours)
    assert len(hr) == len(ho) == 2
    assert [[tuple(t.shape) for t in g] for g in hr] == [[tuple(t.shape) for t in g] for g in ho]
    assert hr[0][0] is ref.actor.model[0].weight if discrete else hr[0][0] is ref.actor.mu[0].weight
    assert hr[0][1] is ref.critic.model[0].weight


def test_integration_patch_rebinds_the_example_imports():
    """INTEGRATION.md's patch for xuance/torch/agents/__init__.py rebinds the module attributes the example imports
    (`from xuance.torch.agents import PPOCLIP_Agent, get_total_iters`, ppo_mujoco.py:61) besides REGISTRY, so the
    unmodified example reaches the device agent.  Applied here to the imported reference module (this container)."""
    if not os.path.isdir("/root/reference"):
        pytest.skip("reference not mounted")
    from tests.golden.ref_loader import import_reference
    import_reference()
    import xuance.torch.agents as ref_agents
    import xuanpolicy_amd.agents as amd
    src = open(os.path.join(REPO, "INTEGRATION.md")).read()
    block = src.split("```python\n# xuance/torch/agents/__init__.py", 1)[1].split("```", 1)[0].split("\n", 1)[1]
    saved = {k: getattr(ref_agents, k) for k in ("PPOCLIP_Agent", "A2C_Agent", "get_total_iters")}
    saved_reg = dict(ref_agents.REGISTRY)
    try:
        exec(compile(block, "INTEGRATION.md", "exec"), ref_agents.__dict__)
        from xuance.torch.agents import A2C_Agent, PPOCLIP_Agent, get_total_iters   # the example's import line
        assert PPOCLIP_Agent is amd.PPOCLIP_Agent and A2C_Agent is amd.A2C_Agent
        assert get_total_iters is amd.get_total_iters
        assert ref_agents.REGISTRY["PPO_Clip"] is amd.PPOCLIP_Agent and ref_agents.REGISTRY["A2C"] is amd.A2C_Agent
    finally:
        for k, v in saved.items():
            setattr(ref_agents, k, v)
        ref_agents.REGISTRY.clear()
        ref_agents.REGISTRY.update(saved_reg)
