"""Drop-in module for the reference's top-level `utils` (ScalarTransforms, get_class,
torch_activation_map)."""
from mzba.scalar import ScalarTransforms, get_class, torch_activation_map  # noqa: F401
