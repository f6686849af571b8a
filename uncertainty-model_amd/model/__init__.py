"""Drop-in ``model`` package (reference model/__init__.py:1-2) backed by the
umamd HIP kernels.  ``Model`` is an alias of ``RandomlyConnectedModel``
(BASELINE north_star names ``model.model.Model``)."""
from .model import RandomlyConnectedModel, Model  # noqa: F401
from .discriminator import RandomDiscriminator  # noqa: F401
