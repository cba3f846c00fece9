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
