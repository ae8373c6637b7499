"""paddle.cost_model (reference: python/paddle/cost_model/cost_model.py)."""
from .cost_model import CostModel, CostData  # noqa: F401

__all__ = ['CostModel']
