"""models/base_models.py surface -> mauv.models (HIP engine)."""
from mauv.models import ResNet50Custom, Identity, AdditiveAttention, MultiModalModel  # noqa: F401
