"""`xuance.torch.agents` (agents/__init__.py:68-111, agent.py:144-145) for PPO_Clip / A2C."""
from ..agents import REGISTRY, A2C_Agent, Agent, PPOCLIP_Agent, get_total_iters  # noqa: F401
