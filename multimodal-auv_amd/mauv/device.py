"""Model placement with the reference's signatures (utils/device.py:6-81).

The reference wraps the tri-modal model in ``nn.DataParallel`` when several devices are given
(utils/device.py:19): one process drives every GPU, replicating all parameters and buffers
into each replica on every forward call.  mauv's engine writes parameter gradients straight
into its gradient arena, which DataParallel's replicate / reduce-add cannot see, so multi-GPU
here is one process per GPU over RCCL:

* launched by ``torchrun --nproc-per-node N script.py`` (WORLD_SIZE > 1 in the environment),
  ``move_model_to_device`` joins the process group (backend "nccl" = RCCL; initialised here
  when the script did not), places every model on this rank's GPU (``cuda:LOCAL_RANK``,
  whatever device the script passed) and wraps the multimodal model in
  ``mauv.ddp.DistributedMC`` (gradient all-reduce over xGMI, MC-sharded prediction) — the
  reference's Examples run unchanged, one rank per GPU, each rank's loader supplying its own
  batches (global batch = ranks x batch size);
* a single process asked to spread a mauv model over several devices raises, saying how to
  launch it instead (the reference's tests assert the DataParallel call for their own dummy
  modules — foreign modules still get ``nn.DataParallel`` as in the reference).
"""
import logging
import os

import torch
import torch.distributed as dist
import torch.nn as nn


def _is_mauv(model):
    from .layers import is_bayesian
    return any(is_bayesian(m) for m in model.modules())


def _world():
    return int(os.environ.get("WORLD_SIZE", "1"))


def distributed_device():
    """This rank's device under torchrun (joins the RCCL process group on first use), else
    None."""
    if _world() <= 1 and not (dist.is_available() and dist.is_initialized()):
        return None
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    if not dist.is_initialized():
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=dev)
        logging.info(f"mauv: joined the RCCL process group as rank {dist.get_rank()} of "
                     f"{dist.get_world_size()} on {dev}")
    return dev if dist.get_world_size() > 1 else None


def move_model_to_device(model, device, device_ids=None):
    try:
        ddp_dev = distributed_device() if _is_mauv(model) else None
        if ddp_dev is not None:
            model = model.to(ddp_dev)
            if device_ids is not None:   # the reference's multi-GPU model: data parallel
                from .ddp import DistributedMC
                model = DistributedMC(model)
                logging.info(f"mauv: rank {dist.get_rank()} of {dist.get_world_size()} on "
                             f"{ddp_dev} (DistributedMC, RCCL gradient all-reduce)")
            return model
        if device_ids and len(device_ids) > 1:
            if _is_mauv(model):
                raise RuntimeError(
                    f"mauv: single-process multi-GPU (nn.DataParallel over {device_ids}) is not "
                    "supported — the engine writes gradients straight into its arena, which "
                    "DataParallel cannot reduce.  Launch one process per GPU instead: "
                    f"`torchrun --nproc-per-node {len(device_ids)} <script>`; "
                    "move_models_to_device then places each rank on its GPU and wraps the "
                    "multimodal model in mauv.ddp.DistributedMC (RCCL all-reduce over xGMI).")
            model = model.to(device)
            logging.info(f"Using multiple GPUs: {device_ids}")
            return nn.DataParallel(model, device_ids=device_ids)
        model = model.to(device)
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
        if ids is None and use_multigpu_for_multimodal and _world() > 1:
            ids = [primary.index]   # torchrun: data parallel across the ranks
        logging.info(f"Moving models to device(s): {devices}")
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
