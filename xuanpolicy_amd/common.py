"""`xuance.common` names the on-policy path uses (the import-swap surface of INTEGRATION.md):
space2shape (common_tools.py:185-189), the config helpers (common_tools.py:13-83) and the drop-in
buffers (memory_tools.py:143-245, 369-492, 526-560)."""
from .buffer import DummyOnPolicyBuffer, DummyOnPolicyBuffer_Atari  # noqa: F401
from .per import PerOffPolicyBuffer  # noqa: F401
from .runner import get_arguments, get_config, recursive_dict_update  # noqa: F401

EPS = 1e-8


def space2shape(observation_space):
    """common_tools.py:185-189 (Dict spaces map key -> shape)."""
    spaces = getattr(observation_space, "spaces", None)
    if isinstance(spaces, dict):
        return {k: v.shape for k, v in spaces.items()}
    return observation_space.shape


def create_directory(path):
    """common_tools.py:170-176."""
    import os
    os.makedirs(path, exist_ok=True)
