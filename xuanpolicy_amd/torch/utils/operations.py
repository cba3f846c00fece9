"""`xuance.torch.utils.operations.set_seed` (operations.py:17-22)."""
from ...runner import set_seed  # noqa: F401
