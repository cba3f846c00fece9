"""`xuance.torch.runners` (runner_drl.py:15-134)."""
from ..runner import REGISTRY, Runner_DRL  # noqa: F401
