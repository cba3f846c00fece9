"""xuanpolicy_amd — MI355X (gfx950) native on-policy PPO-Clip / A2C hot path for XuanCe.

The reference's on-policy loop (DummyOnPolicyBuffer + finish_path GAE + PPOCLIP_Learner /
A2C_Learner + the agent's rollout loop) rebuilt as a device-resident pipeline: hand-written HIP
kernels behind a C ABI (include/xuanpolicy_amd.h, libxuanpolicy_amd.so) for GAE, the fused loss,
minibatch gather, running normalisation, action sampling, the synthetic env step and the per-step
bookkeeping; PyTorch-ROCm for the actor-critic GEMMs; RCCL for the data-parallel gradient all-reduce.

The native library is loaded on first use and every op raises if it is missing: there is no CPU path.
"""
import torch  # noqa: F401  (HIP runtime must be mapped before the native library)

from ._lib import XpaError, build_library, load as load_library  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # Lazy submodule access keeps `import xuanpolicy_amd` cheap and CPU-safe.
    import importlib
    if name in ("ops", "buffer", "learners", "agents", "policies", "envs", "distributed", "config", "runner", "common",
                "environment"):
        return importlib.import_module("." + name, __name__)
    if name in ("get_arguments", "get_runner"):   # `from xuance import get_arguments, get_runner`
        return getattr(importlib.import_module(".runner", __name__), name)
    raise AttributeError(name)
