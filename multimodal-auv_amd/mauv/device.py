"""Model placement with the reference's signatures (utils/device.py:6-81).

The reference wraps the tri-modal model in ``nn.DataParallel`` when several devices are given
(utils/device.py:19).  mauv's engine writes parameter gradients straight into its gradient
arena, which DataParallel's replicate/reduce-add cannot see, so multi-GPU here is one process
per GPU: launch with torchrun and wrap with ``mauv.ddp.DistributedMC`` (RCCL all-reduce over
xGMI).  Asking for several device ids in one process keeps the model on the first one and
says so.
"""
import logging

import torch.nn as nn


def move_model_to_device(model, device, device_ids=None):
    try:
        model = model.to(device)
        if device_ids and len(device_ids) > 1:
            logging.warning(
                f"mauv: single-process multi-GPU (nn.DataParallel over {device_ids}) is not used; "
                "run one process per GPU (torchrun) and wrap with mauv.ddp.DistributedMC. "
                f"Model kept on {device}.")
        else:
            logging.info(f"Using single device: {device}")
        return model
    except Exception as e:
        logging.error(f"Error moving model to device: {e}", exc_info=True)
        raise


def move_models_to_device(models_dict, devices, use_multigpu_for_multimodal=True):
    try:
        primary = devices[0]
        ids = [d.index for d in devices] if use_multigpu_for_multimodal and len(devices) > 1 \
            else None
        for name, model in models_dict.items():
            if model is None:
                continue
            models_dict[name] = move_model_to_device(
                model, primary, ids if "multimodal_model" in name else None)
        return models_dict
    except Exception as e:
        logging.error(f"Error moving models to devices: {e}", exc_info=True)
        raise


def check_model_devices(model, expected_device):
    for name, param in model.named_parameters():
        if param.device != expected_device:
            logging.warning(f"Param {name} is on {param.device}, expected {expected_device}")
            return False
    logging.info("All model parameters are on the expected device.")
    return True
