"""bayesian_torch.layers -> mauv reparameterisation layers (same parameter names)."""
from mauv.layers import Conv2dReparameterization, LinearReparameterization  # noqa: F401
