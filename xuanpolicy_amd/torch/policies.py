"""`xuance.torch.policies` (gaussian.py:54-77, categorical.py:61-85) for the on-policy path."""
from ..policies import REGISTRY, Categorical_AC_Policy, Gaussian_AC_Policy  # noqa: F401
