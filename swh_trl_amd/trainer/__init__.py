"""Drop-in trainer classes (reference: trl/trainer/grpo_trainer.py, ppo_trainer.py)."""
from .grpo_config import GRPOConfig
from .grpo_trainer import GRPOTrainer
from .ppo_config import PPOConfig
from .ppo_trainer import PPOTrainer

__all__ = ["GRPOConfig", "GRPOTrainer", "PPOConfig", "PPOTrainer"]
