"""`xuance.torch.utils` names used by the on-policy examples."""
from ...policies import (ActivationFunctions, CategoricalDistribution, DiagGaussianDistribution,  # noqa: F401
                         InitializeFunctions, NormalizeFunctions, cnn_block, mlp_block)
from .operations import set_seed  # noqa: F401
