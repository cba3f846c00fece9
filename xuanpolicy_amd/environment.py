"""`xuance.environment.make_envs` (environment/__init__.py:36-99) for the envs of this path: the
device-resident SynthBox / SynthAtari vector envs (BASELINE.json configs).  Host VecEnvs with the
reference's step contract can be handed to the agents directly."""
from .runner import make_envs  # noqa: F401
