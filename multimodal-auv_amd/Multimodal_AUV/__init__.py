"""Drop-in for sams-tom/Multimodal-AUV's hot path, backed by mauv (MI355X HIP kernels).

Same import paths as the reference for the on-path modules:
  Multimodal_AUV.models.{base_models,model_utils}, Multimodal_AUV.train.{multimodal,unimodal,
  loop_utils,checkpointing}, Multimodal_AUV.inference.predictors, Multimodal_AUV.utils.device
Off-path modules (data, config, data_preparation, functions, Examples) stay the reference's
own: set MAUV_REFERENCE_PKG=/path/to/reference/src/Multimodal_AUV and they resolve from
there (this package's modules take precedence).  See INTEGRATION.md.
"""
import logging
import os

_ref = os.environ.get("MAUV_REFERENCE_PKG")
if _ref and os.path.isdir(_ref) and _ref not in __path__:
    __path__.append(_ref)

__version__ = "0.1.0+mauv"
logging.getLogger(__name__).addHandler(logging.NullHandler())
