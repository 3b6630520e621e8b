"""bayesian_torch.models.dnn_to_bnn -> mauv (MOPED conversion, fused KL)."""
from mauv.layers import dnn_to_bnn  # noqa: F401
from mauv.kl import get_kl_loss  # noqa: F401
