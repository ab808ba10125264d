"""Drop-in trainer classes (reference: trl/trainer/grpo_trainer.py, ppo_trainer.py)."""
from .grpo_config import GRPOConfig
from .grpo_trainer import GRPOTrainer

__all__ = ["GRPOConfig", "GRPOTrainer"]
