"""Command-line runner for the on-policy path, as XuanCe's `get_runner(...).run()/.benchmark()` scripts:

    python examples/run_on_policy.py --method ppo --env synthbox --env-id SynthBox-v0 \
        --config examples/ppo_synthbox_config.yaml --benchmark 1

The reference's own examples (examples/ppo/ppo_mujoco.py, ppo_atari.py) run unchanged apart from the
`xuance` -> `xuanpolicy_amd` import swap."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser("xuanpolicy_amd on-policy runner")
    p.add_argument("--method", default="ppo")
    p.add_argument("--env", default="synthbox")
    p.add_argument("--env-id", default="SynthBox-v0")
    p.add_argument("--config", default=None)
    p.add_argument("--device", default="cuda:0")
    p.add_argument("--test", type=int, default=0)
    p.add_argument("--benchmark", type=int, default=0)
    a = p.parse_args()
    from xuanpolicy_amd import get_runner
    runner = get_runner(a.method, a.env, a.env_id, a.config, a, is_test=bool(a.test))
    if a.benchmark:
        runner.benchmark()
    else:
        runner.run()


if __name__ == "__main__":
    main()
