"""mauv — MI355X-native Monte-Carlo Bayesian tri-modal encoder (Multimodal-AUV hot path).

Host side of the drop-in: PyTorch-ROCm modules whose compute runs entirely in
libmauv_hip.so (hand-written gfx950 HIP kernels behind the C-ABI of include/mauv.h).
"""
from ._lib import lib, MauvError  # noqa: F401  (fails loudly if the HIP library is missing)

__version__ = "0.1.0"
