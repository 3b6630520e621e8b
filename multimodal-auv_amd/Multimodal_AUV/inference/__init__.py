"""Multimodal_AUV.inference (mauv drop-in); the reference's other inference modules resolve through
MAUV_REFERENCE_PKG (see the top package)."""
from .. import _extend_path

__path__ = _extend_path(__path__, "inference")
