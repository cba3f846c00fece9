"""`xuance.torch.representations` (mlp.py:6-51, cnn.py:45-93) for the on-policy path."""
from ..policies import AC_CNN_Atari, Basic_Identical, Basic_MLP  # noqa: F401
from ..policies import REGISTRY_Representation as REGISTRY  # noqa: F401
