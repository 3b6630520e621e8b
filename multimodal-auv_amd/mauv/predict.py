"""MC inference with the reference's call surface (inference/predictors.py:9-97).

``multimodal_predict_and_save`` writes the same CSV (``Image Name, Predicted Class,
Predictive Uncertainty, Aleatoric Uncertainty``) with the same maths (softmax per pass,
unbiased variance over the MC samples averaged over classes, aleatoric = mean entropy with
eps 1e-7, class = argmax of the mean probability) — but the ``num_mc_samples`` passes run as
batched launches (``mc_forward``, chunked to fit HBM) and the statistics are one fused
reduction (mauv_mc_stats / mauv_mc_finalize) whose partial sums all-reduce across ranks for
MC-sharded multi-GPU inference.

Numerics: the reference autocasts to fp16 on CUDA (predictors.py:55); mauv runs the model's
compute dtype (fp32 by default) and always reduces in fp32/fp64.
"""
import csv
import logging

import torch
import torch.distributed as dist

from . import mchead
from .kl import unwrap


def mc_chunk(model, batch_size, num_mc, budget_bytes=None):
    """How many MC samples to batch per launch for inference (activation memory bound)."""
    core = unwrap(model)
    if budget_bytes is None:
        budget_bytes = getattr(core, "mc_infer_budget_bytes", 64 << 30)
    # peak live activations ≈ 4 x the largest NHWC tensor (stem out, 64 x H/2 x W/2) per
    # trunk image, fp32; sonar tiles are 256 px in the reference
    per_sample = 4 * 4 * 64 * 128 * 128 * batch_size
    return max(1, min(num_mc, int(budget_bytes // max(per_sample, 1))))


def local_mc_count(num_mc, rank, world):
    """MC samples this rank draws when ``num_mc`` are sharded over ``world`` ranks."""
    return num_mc // world + (1 if rank < num_mc % world else 0)


def mc_statistics(model, inputs, bathy, sss, num_mc, eps_h=1e-7, eps_pred=1e-8, chunk=None,
                  group=None):
    """Fused MC statistics for one batch; with ``group`` (torch.distributed), the MC samples
    are sharded across ranks (each rank: full batch, ~num_mc/world samples; BN statistics
    stay per-sample exactly as in the reference) and the sums all-reduced once."""
    B = inputs.shape[0]
    rank, world = (dist.get_rank(group), dist.get_world_size(group)) if group is not None \
        else (0, 1)
    local = local_mc_count(num_mc, rank, world)
    chunk = chunk or mc_chunk(model, B, max(local, 1))
    core = model if hasattr(model, "mc_forward") else unwrap(model)
    sums = None
    done = 0
    while done < local:
        g = min(chunk, local - done)
        logits = core.mc_forward(inputs, bathy, sss, g)
        sums = mchead.mc_stats(logits, eps_h, sums)
        done += g
        del logits
    C = unwrap(model).fc2.out_features
    if sums is None:
        sums = torch.zeros(B, 2 * C + 1, dtype=torch.float64, device=inputs.device)
    if group is not None:
        dist.all_reduce(sums, group=group)
    return mchead.mc_finalize(sums, num_mc, C, eps_pred)


def multimodal_predict_and_save(multimodal_model, dataloader, device, csv_path,
                                num_mc_samples=10, sss_patch_type="", channel_patch_type="",
                                model_type="multimodal"):
    """inference/predictors.py:9-97 (model kept in .train(): BN uses batch statistics)."""
    multimodal_model.train()
    logging.info(f"CSV will be saved to: {csv_path}")
    with open(csv_path, mode="w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Image Name", "Predicted Class", "Predictive Uncertainty",
                    "Aleatoric Uncertainty"])
        with torch.no_grad():
            for batch_idx, (inputs, bathy, sss, image_name) in enumerate(dataloader):
                inputs = inputs.to(device, non_blocking=True)
                bathy = bathy.to(device, non_blocking=True)
                sss = sss.to(device, non_blocking=True)
                if hasattr(unwrap(multimodal_model), "mc_forward"):
                    st = mc_statistics(multimodal_model, inputs, bathy, sss, num_mc_samples)
                    pred, var, alea = st["pred"], st["var"], st["aleatoric"]
                else:  # foreign model: reference sequential loop
                    P = torch.stack([torch.softmax(multimodal_model(inputs, bathy, sss), 1)
                                     for _ in range(num_mc_samples)])
                    var = torch.var(P, dim=0).mean(dim=1)
                    alea = torch.mean(-torch.sum(P * torch.log(P + 1e-7), dim=-1), dim=0)
                    pred = torch.argmax(P.mean(0), dim=1)
                pred, var, alea = pred.cpu().tolist(), var.cpu().tolist(), alea.cpu().tolist()
                for i in range(inputs.size(0)):
                    name = image_name[i] if isinstance(image_name, (list, tuple)) else image_name
                    w.writerow([name, pred[i], var[i], alea[i]])
    logging.info("Completed: multimodal_predict_and_save")
