"""Checkpoint format compatibility (train/checkpointing.py:7-112).

State dicts use bayesian-torch's key names (``...conv1.mu_kernel``, ``fc2.mu_weight`` ...), so
reference checkpoints load into mauv models and vice versa.  Loading is always
``weights_only=True``.
"""
import logging
import os

import torch


def save_model(model, csv_path, patch_type):
    """<dirname(dirname(csv_path))>/models/bayesian_model_type{patch_type}.pth"""
    try:
        models_dir = os.path.join(os.path.dirname(os.path.dirname(csv_path)), "models")
        os.makedirs(models_dir, exist_ok=True)
        path = os.path.join(models_dir, f"bayesian_model_type{patch_type}.pth")
        torch.save(_unwrap(model).state_dict(), path)
        logging.info(f"Model saved successfully to {path}")
    except Exception as e:
        logging.error(f"Error saving model: {e}", exc_info=True)


def _unwrap(model):
    from .kl import unwrap
    return unwrap(model)


def remap_keys(state_dict, model_keys, num_classes=None):
    """Key rewrites the reference applies before loading (Example_Inference_model.py:83-108,
    checkpointing.py:79-100): strip ``module.``; ``*_model_feat.model.`` -> ``*_model_feat.``;
    drop ``fc2.*`` when its shape does not match (num_classes != 7).  Returns
    (new_state_dict, skipped_descriptions)."""
    out, skipped = {}, []
    for k, v in state_dict.items():
        km = k[len("module."):] if k.startswith("module.") else k
        for feat in ("image_model_feat", "bathy_model_feat", "sss_model_feat"):
            km = km.replace(f"{feat}.model.", f"{feat}.")
        if km not in model_keys:
            skipped.append(f"  - Key '{k}' (mapped to '{km}') as it is not found in the current model.")
            continue
        if tuple(v.shape) != tuple(model_keys[km]):
            skipped.append(f"  - Key '{k}' (mapped to '{km}') due to shape mismatch: "
                           f"checkpoint has {tuple(v.shape)}, model has {tuple(model_keys[km])}")
            continue
        out[km] = v
    return out, skipped


def load_and_fix_state_dict(model, model_path, device):
    """Tolerant loader; returns a bare bool like the reference (checkpointing.py:108,112)."""
    if not os.path.exists(model_path):
        logging.warning(f"Model checkpoint not found at: {model_path}. Skipping load.")
        return False
    try:
        sd = torch.load(model_path, map_location=device, weights_only=True)
        target = _unwrap(model)
        keys = {k: v.shape for k, v in target.state_dict().items()}
        new_sd, skipped = remap_keys(sd, keys)
        target.load_state_dict(new_sd, strict=False)
        logging.info("Model state_dict loaded successfully.")
        logging.info(f"Skipped layers: {skipped}")
        return True
    except Exception as e:
        logging.error(f"An unexpected error occurred while loading state_dict for {model_path}: {e}",
                      exc_info=True)
        return False
