"""Multimodal_AUV.models (mauv drop-in); the reference's other models modules resolve through
MAUV_REFERENCE_PKG (see the top package)."""
from .. import _extend_path

__path__ = _extend_path(__path__, "models")
