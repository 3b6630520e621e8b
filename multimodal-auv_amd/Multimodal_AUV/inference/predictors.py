"""inference/predictors.py surface -> mauv.predict (batched MC + fused uncertainty)."""
from mauv.predict import multimodal_predict_and_save, mc_statistics  # noqa: F401
