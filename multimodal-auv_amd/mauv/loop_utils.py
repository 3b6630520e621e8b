"""Epoch drivers and optimiser factory with the reference's signatures (train/loop_utils.py).

* ``define_optimizers_and_schedulers``      loop_utils.py:13-63 (CE + 4 Adam + 4 StepLR; Adam
                                            is mauv.optim.FusedAdam — one HIP launch per step —
                                            for models on a ROCm device, torch's otherwise)
* ``train_and_evaluate_unimodal_model``     loop_utils.py:65-159 (epochs ``range(1, n)``)
* ``train_and_evaluate_multimodal_model``   loop_utils.py:162-250 (scheduler stepped after
                                            training AND after evaluation, as the reference)
"""
import logging
import os

import torch.nn as nn
import torch.optim as optim

from .optim import FusedAdam
from .train import (train_unimodal_model, evaluate_unimodal_model, train_multimodal_model,
                    evaluate_multimodal_model)

_MODEL_KEYS = ("image_model", "bathy_model", "sss_model", "multimodal_model")


def define_optimizers_and_schedulers(models_dict, optimizer_params=None, scheduler_params=None,
                                     criterion_type="cross_entropy"):
    if criterion_type != "cross_entropy":
        logging.error(f"Unsupported criterion type provided: {criterion_type}")
        raise ValueError(f"Unsupported criterion: {criterion_type}")
    criterion = nn.CrossEntropyLoss()
    def adam(model, kw):
        params = list(model.parameters())
        on_gpu = all(p.is_cuda for p in params)
        return (FusedAdam if on_gpu else optim.Adam)(params, **kw)
    optimizers = {k: adam(models_dict[k], optimizer_params[k]) for k in _MODEL_KEYS}
    schedulers = {k: optim.lr_scheduler.StepLR(optimizers[k], **scheduler_params[k])
                  for k in optimizers}
    return criterion, optimizers, schedulers


def train_and_evaluate_unimodal_model(model, train_loader, test_loader, criterion, optimizer,
                                      scheduler, num_epochs, device, model_name, save_dir,
                                      num_mc, sum_writer):
    logging.info(f"Training started for unimodal model: {model_name} ({num_epochs} epochs, "
                 f"num_mc={num_mc})")
    for epoch in range(1, num_epochs):
        train_accuracy, train_loss = train_unimodal_model(
            model=model, dataloader=train_loader, criterion=criterion, optimizer=optimizer,
            epoch=epoch, total_num_epochs=num_epochs, num_mc=num_mc, device=device,
            model_type=model_name, csv_path=os.path.join(save_dir, f"{model_name}.csv"),
            sum_writer=sum_writer)
        val_accuracy = evaluate_unimodal_model(
            model=model, dataloader=test_loader, device=device, epoch=epoch,
            total_num_epochs=num_epochs, num_mc=num_mc, model_type=model_name,
            csv_path=os.path.join(save_dir, f"{model_name}_evaluate.csv"))
        scheduler.step()
        sum_writer.add_scalar("train/loss/epoch", train_loss, epoch)
        sum_writer.add_scalar("val/accuracy/epoch", val_accuracy, epoch)
    logging.info(f"Training completed for unimodal model: {model_name}")


def train_and_evaluate_multimodal_model(train_loader, test_loader, multimodal_model, criterion,
                                        optimizer, lr_scheduler, num_epochs, num_mc, device,
                                        model_type, bathy_patch_type, sss_patch_type, csv_path,
                                        sum_writer):
    logging.info(f"Multimodal training: {model_type}, bathy={bathy_patch_type}, "
                 f"sss={sss_patch_type}, epochs={num_epochs}, num_mc={num_mc}")
    try:
        os.makedirs(csv_path, exist_ok=True)
    except OSError as e:
        logging.error(f"Failed to create CSV output directory {csv_path}: {e}")
    for epoch in range(num_epochs):
        train_loss, train_accuracy = train_multimodal_model(
            multimodal_model=multimodal_model, dataloader=train_loader, criterion=criterion,
            optimizer=optimizer, epoch=epoch, total_num_epochs=num_epochs, device=device,
            model_type=model_type, num_mc=num_mc, bathy_patch_type=bathy_patch_type,
            sss_patch_type=sss_patch_type,
            csv_path=os.path.join(csv_path, "multimodal_training.csv"), sum_writer=sum_writer)
        lr_scheduler.step()
        val_accuracy = evaluate_multimodal_model(
            multimodal_model=multimodal_model, dataloader=test_loader, device=device,
            epoch=epoch, total_num_epochs=num_epochs, num_mc=num_mc,
            csv_path=os.path.join(csv_path, "multimodal_test.csv"),
            bathy_patch_type=bathy_patch_type, sss_patch_type=sss_patch_type,
            model_type=model_type)
        lr_scheduler.step()
        sum_writer.add_scalar("train/loss/epoch", train_loss, epoch)
        sum_writer.add_scalar("val/accuracy/epoch", val_accuracy, epoch)
    logging.info(f"Finished multimodal training C:{bathy_patch_type}, S:{sss_patch_type}")
