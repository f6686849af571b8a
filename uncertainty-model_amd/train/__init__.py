"""Drop-in ``train`` package (reference train/__init__.py:1-3)."""
from . import transforms  # noqa: F401
from .train import train_model  # noqa: F401
from .evaluate import evaluate_model  # noqa: F401
