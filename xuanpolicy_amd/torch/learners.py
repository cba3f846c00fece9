"""`xuance.torch.learners` (learner.py:10-52, ppoclip_learner.py, a2c_learner.py)."""
from ..learners import REGISTRY, A2C_Learner, Learner, PPOCLIP_Learner  # noqa: F401
