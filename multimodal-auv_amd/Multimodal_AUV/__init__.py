"""Drop-in for sams-tom/Multimodal-AUV's hot path, backed by mauv (MI355X HIP kernels).

Same import paths as the reference for the on-path modules:
  Multimodal_AUV.models.{base_models,model_utils}, Multimodal_AUV.train.{multimodal,unimodal,
  loop_utils,checkpointing}, Multimodal_AUV.inference.predictors, Multimodal_AUV.utils.device
Off-path modules (data, config, data_preparation, functions, Examples, inference.inference_data)
stay the reference's own: set MAUV_REFERENCE_PKG=/path/to/reference/src/Multimodal_AUV and they
resolve from there — in this package and in every drop-in subpackage (this package's modules
take precedence).  The reference's top-level API (`__init__.py:5-10`: run_auv_inference,
run_auv_retraining, run_auv_preprocessing, run_AUV_training_from_scratch) is re-exported lazily
from its `functions.functions`, which then runs on the drop-in modules.  See INTEGRATION.md.
"""
import logging
import os

_REF_API = ("run_auv_inference", "run_auv_retraining", "run_auv_preprocessing",
            "run_AUV_training_from_scratch")


def _reference_dir():
    ref = os.environ.get("MAUV_REFERENCE_PKG")
    return ref if ref and os.path.isdir(ref) else None


def _extend_path(path, sub=""):
    """Append the reference's same-named package directory to a drop-in package's __path__."""
    ref = _reference_dir()
    if ref:
        d = os.path.join(ref, sub) if sub else ref
        if os.path.isdir(d) and d not in path:
            path.append(d)
    return path


_extend_path(__path__)


def __getattr__(name):
    # PEP 562: `from Multimodal_AUV import run_auv_inference` (the reference's README usage)
    if name in _REF_API:
        if _reference_dir() is None:
            raise ImportError(f"Multimodal_AUV.{name} is the reference's orchestration API "
                              "(functions/functions.py); set MAUV_REFERENCE_PKG to the "
                              "reference's src/Multimodal_AUV to use it on the mauv drop-in")
        from .functions import functions as _f
        val = getattr(_f, name)
        globals()[name] = val
        return val
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


__all__ = list(_REF_API) if _reference_dir() else []
__version__ = "0.1.0+mauv"
logging.getLogger(__name__).addHandler(logging.NullHandler())
