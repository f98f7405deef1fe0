from .learning_rate import build_learning_rate, warmup_factor_at_step
from .optimizer import MomentumSGD, param_groups

__all__ = ["build_learning_rate", "warmup_factor_at_step", "MomentumSGD", "param_groups"]
