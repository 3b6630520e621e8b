"""MC training / evaluation loops with the reference's call surface.

Signatures, return values, CSV rows, KL weighting and skip rules follow
``train/multimodal.py`` and ``train/unimodal.py``; the difference is inside the batch:

* the ``num_mc`` stochastic forwards run as ONE batched pass (``model.mc_forward``) instead of
  a Python loop of single forwards (multimodal.py:107-118, unimodal.py:127-130);
* the KL term is computed once per batch (it does not depend on the MC sample — the reference
  recomputes the identical value ``num_mc`` times and averages);
* mean-over-MC + cross-entropy is one fused kernel; the NaN/Inf gradient guard
  (multimodal.py:141) is one fused scan over the flat gradient arena + one host sync instead
  of ~700 per-tensor syncs.

Models without ``mc_forward`` (e.g. the reference tests' dummy modules, which run on
``device='cpu'``) run the reference's sequential loop and its torch maths unchanged; the fused
kernels are used only on ROCm tensors (a host pointer must never reach a HIP kernel).
"""
import csv
import logging
import os
from pathlib import Path

import numpy as np
import torch
import torch.nn as nn

from .kl import get_kl_loss, unwrap
from . import mchead


def kl_weight_for(epoch, total_num_epochs):
    return (2 ** (epoch + 1)) / (2 ** total_num_epochs)  # multimodal.py:80, unimodal.py:71


def _is_plain_ce(criterion):
    return (type(criterion) is nn.CrossEntropyLoss and criterion.weight is None
            and criterion.reduction == "mean" and criterion.ignore_index == -100
            and float(getattr(criterion, "label_smoothing", 0.0)) == 0.0)


def mc_logits(model, num_mc, *inputs):
    """[num_mc, B, C]: batched on mauv models, the reference's sequential loop otherwise."""
    core = unwrap(model)
    if hasattr(core, "mc_forward"):
        return model.mc_forward(*inputs, num_mc) if hasattr(model, "mc_forward") \
            else core.mc_forward(*inputs, num_mc)
    if isinstance(model, torch.nn.parallel.DistributedDataParallel):
        model = model.module
    return torch.stack([model(*inputs) for _ in range(num_mc)])


def _grads_finite(model):
    st = unwrap(model).__dict__.get("_mauv_state")
    if st is not None and st.arena is not None and all(
            p.grad is None or p.grad.data_ptr() == v.data_ptr()
            for p, v in zip(st.arena.params, st.arena.views)):
        return mchead.all_finite(st.arena.flat)
    grads = [p.grad for p in model.parameters() if p.grad is not None]
    if not grads:
        return True
    if all(g.is_cuda for g in grads):
        return mchead.all_finite(grads)
    # foreign model on the host: the reference's per-tensor scan (multimodal.py:141)
    return not any(torch.isnan(g).any() or torch.isinf(g).any() for g in grads)


def _all_ranks(model, flag):
    """A DistributedMC model agrees on a per-rank decision (logical AND over ranks), so that
    every rank skips the same batches and the gradient all-reduces stay paired."""
    return model.all_ranks(flag) if hasattr(model, "all_ranks") else flag


def mc_eval_stats(logits, labels, eps_pred, eps_h):
    """CE of the MC-mean logits, argmax, and the MC uncertainty statistics of one eval batch
    (multimodal.py:287-310 / unimodal.py:285-300): fused kernels for ROCm logits, the
    reference's torch maths for a foreign model's host logits."""
    N, _, C = logits.shape
    if logits.is_cuda:
        ce, _, predicted = mchead.mc_mean_ce(logits, labels)
        st = mchead.mc_finalize(mchead.mc_stats(logits, eps_h), N, C, eps_pred)
        return ce, predicted, st
    out_mean = logits.mean(0)
    ce = torch.nn.functional.cross_entropy(out_mean, labels)
    predicted = torch.max(out_mean, 1)[1]
    P = torch.softmax(logits.float(), dim=2)
    mean_p = P.mean(0)
    st = dict(mean_prob=mean_p,
              predictive_entropy=-torch.sum(mean_p * torch.log(mean_p + eps_pred), dim=1),
              aleatoric=torch.mean(-torch.sum(P * torch.log(P + eps_h), dim=2), dim=0),
              var=torch.var(P, dim=0).mean(dim=1), pred=torch.argmax(mean_p, dim=1))
    return ce, predicted, st


def mc_loss(model, inputs_tuple, labels, criterion, num_mc, batch_size, kl_w):
    """Forward part of one training batch -> (loss, output_mean, predicted, ce, scaled_kl)."""
    logits = mc_logits(model, num_mc, *inputs_tuple)
    kl = get_kl_loss(model)
    if _is_plain_ce(criterion) and logits.is_cuda:
        ce, output, predicted = mchead.mc_mean_ce(logits, labels)
    else:
        output = mchead.mc_mean(logits) if logits.is_cuda else logits.mean(0)
        ce = criterion(output, labels)
        predicted = torch.max(output.detach(), 1)[1]
    scaled_kl = kl / batch_size * kl_w if kl is not None else torch.zeros((), device=ce.device)
    return ce + scaled_kl, output, predicted, ce, scaled_kl


def _step_gate(model, optimizer, loss):
    """The device MauvStepGate when the batch can be decided on the device: a mauv engine model
    whose gradients live in its arena, stepped by FusedAdam over exactly its parameters."""
    from .optim import FusedAdam
    if not isinstance(optimizer, FusedAdam) or not loss.is_cuda:
        return None
    st = unwrap(model).__dict__.get("_mauv_state")
    if st is None or not all(p.requires_grad for p in st.params):
        return None
    return optimizer.gate(st.params, loss.device)


def _batch_finite(loss, inputs_tuple, counter=None):
    """Device bool: the reference would see a finite loss (multimodal.py:133).  Besides the
    loss itself, any non-finite input pixel counts: with BatchNorm in train mode one NaN / Inf
    pixel makes every logit of the reference's batch NaN (torch's ReLU propagates NaN), while
    the fused kernels' ReLU (x > 0 ? x : 0) would zero a NaN channel and hand back a finite
    loss over non-finite gradients.  ``counter``: int32 device scratch word."""
    from . import ops
    ok = torch.isfinite(loss.detach()).reshape(1)
    ins = [t for t in inputs_tuple if t.is_cuda and t.dtype == torch.float32 and
           t.is_contiguous()]
    if not ins:
        return ok
    if counter is None:
        counter = torch.zeros(1, dtype=torch.int32, device=loss.device)
    else:
        counter.zero_()
    for t in ins:
        ops.nonfinite_count(t, counter)
    return ok & (counter == 0)


def _count_nonfinite(model, counter):
    """Add the number of non-finite gradient blocks of the arena into the device ``counter``
    (the fused form of multimodal.py:141's per-tensor isnan/isinf scan, no host sync)."""
    st = unwrap(model).__dict__["_mauv_state"]
    from . import ops
    ops.nonfinite_count(st.arena.flat, counter)


_MAX_STEPS_AHEAD = 2


def _throttle(model):
    """With no host round trip in a step the host could enqueue steps without bound; it stays
    at most ``_MAX_STEPS_AHEAD`` steps ahead of the GPU (it waits for the end of the step
    before the previous one, so the GPU always has a whole queued step while the host works)."""
    st = unwrap(model).__dict__.get("_mauv_state")
    if st is None or not torch.cuda.is_available():
        return None
    q = st.__dict__.setdefault("step_events", [])
    while len(q) >= _MAX_STEPS_AHEAD:
        q.pop(0).synchronize()
    return q


def mc_train_step(model, inputs_tuple, labels, criterion, optimizer, num_mc, batch_size, kl_w):
    """One reference training batch (multimodal.py:104-146): MC forward, KL, CE, NaN/Inf loss
    skip, backward, NaN/Inf gradient guard, optimizer step + zero_grad.

    For a mauv model stepped by FusedAdam the two skip decisions are taken on the device
    (``MauvStepGate``, adam.hip): the finite-loss flag is written (and MIN-reduced over the
    ranks of a DistributedMC job) before the backward, the gradient arena's non-finite count
    after it, and the Adam kernel steps + zeroes the gradients, takes the batch's gradients
    back out (non-finite loss: the reference never ran that backward), or leaves the arena
    alone (non-finite gradients: no zero_grad, multimodal.py:141-145).  Nothing here waits on
    the GPU; ``ok_loss`` / ``stepped`` come back as device tensors.  Other models and
    optimizers take the host-decided path (None for a skipped batch)."""
    inflight = _throttle(model)
    loss, output, predicted, ce, scaled_kl = mc_loss(model, inputs_tuple, labels, criterion,
                                                     num_mc, batch_size, kl_w)
    gate = _step_gate(model, optimizer, loss)
    if gate is not None:
        from .optim import G_OK_LOSS, G_NONFINITE, G_STEPPED, G_SCRATCH
        ok = gate[G_OK_LOSS:G_OK_LOSS + 1]
        ok.copy_(_batch_finite(loss, inputs_tuple, gate[G_SCRATCH:G_SCRATCH + 1]))
        if hasattr(model, "all_ranks_device"):
            model.all_ranks_device(ok)
        loss.backward()
        if hasattr(model, "allreduce_grads"):  # mauv.ddp.DistributedMC: RCCL all-reduce
            model.allreduce_grads()
        _count_nonfinite(model, gate[G_NONFINITE:G_NONFINITE + 1])
        optimizer.step_gated(gate)
        flags = gate[:G_STEPPED + 1].clone() != 0   # this batch's decisions (device)
        if inflight is not None:
            ev = torch.cuda.Event()
            ev.record()
            inflight.append(ev)
        return dict(loss=loss.detach(), output=output, predicted=predicted, ce=ce.detach(),
                    scaled_kl=scaled_kl.detach(), ok_loss=flags[G_OK_LOSS],
                    stepped=flags[G_STEPPED])
    if not _all_ranks(model, bool(_batch_finite(loss, inputs_tuple).item())):
        logging.warning(f"Skipping batch due to NaN/Inf loss: {loss}")
        return None
    loss.backward()
    if hasattr(model, "allreduce_grads"):  # mauv.ddp.DistributedMC: one RCCL all-reduce
        model.allreduce_grads()
    stepped = _grads_finite(model)   # identical on every rank after the all-reduce
    if stepped:
        optimizer.step()
        optimizer.zero_grad()
    else:
        logging.warning("Skipping optimizer step due to NaN/Inf gradients")
    return dict(loss=loss.detach(), output=output, predicted=predicted, ce=ce.detach(),
                scaled_kl=scaled_kl.detach(), stepped=stepped)


class _TrainEpoch:
    """Per-batch bookkeeping of train_multimodal_model (multimodal.py:133-166) without a host
    round trip on the batch just issued: a batch's loss, correct count and skip decisions are
    read when the NEXT batch has been issued (the GPU is then still busy), so the host never
    idles the GPU.  Batches whose loss was non-finite are not counted or logged, exactly as the
    reference's ``continue``; the running figures, TensorBoard scalars and log lines come out in
    the reference's order and values."""

    def __init__(self, epoch, sum_writer):
        self.epoch, self.writer = epoch, sum_writer
        self.total_loss, self.correct, self.total = 0.0, 0, 0
        self.last = None
        self.pending = []

    def add(self, i, r, labels):
        keep = ("loss", "ce", "scaled_kl", "ok_loss", "stepped")
        r = dict({k: r[k] for k in keep if k in r},
                 n_correct=(r["predicted"] == labels).sum(), n=labels.size(0))
        self.pending.append((i, r))
        if len(self.pending) > 1:
            self._settle(self.pending.pop(0))

    def flush(self):
        while self.pending:
            self._settle(self.pending.pop(0))

    def _settle(self, item):
        i, r = item
        if "ok_loss" in r and not bool(r["ok_loss"]):
            logging.warning(f"Skipping batch {i} due to NaN/Inf loss: {r['loss']}")
            return
        if "ok_loss" in r and not bool(r["stepped"]):   # (the host-decided path warned already)
            logging.warning("Skipping optimizer step due to NaN/Inf gradients")
        lv = r["loss"].item()
        self.total_loss += lv
        self.correct += int(r["n_correct"].item())
        self.total += r["n"]
        self.last = r
        self.writer.add_scalar("Loss/train", lv, i)
        logging.info(f"[Epoch {self.epoch} | Batch {i}] Loss: {lv:.4f}, "
                     f"Accuracy: {self.correct / max(self.total, 1):.4f}")


def loop_device(model, device):
    """The device a loop moves its batches to.  Under torchrun the mauv model sits on this
    rank's GPU (mauv.device.move_model_to_device) while the reference scripts keep passing
    ``devices[0]`` to the loops (Example_training_from_scratch.py:93): the batches follow the
    model, as they must for its kernels.  Foreign models keep the caller's device."""
    core = unwrap(model)
    if hasattr(core, "mc_forward"):
        for p in core.parameters():
            if p.is_cuda and p.device != torch.device(device):
                return p.device
            break
    return device


def is_writer(model):
    """Only rank 0 of a DistributedMC job writes CSV rows, plots and checkpoints; the other
    ranks run the same batches and collectives."""
    return not (getattr(model, "_mauv_wrapper", False) and getattr(model, "world", 1) > 1
                and getattr(model, "rank", 0) != 0)


def sum_ranks(model, values):
    """Element-wise sum of a list of floats over the ranks of a DistributedMC job (identity
    on one process)."""
    if hasattr(model, "sum_ranks") and getattr(model, "world", 1) > 1:
        return model.sum_ranks(values)
    return list(values)


def _tile_to(t, device, optical=False):
    """Move one image batch to the device; decoded uint8 HWC tiles (4x fewer bytes over PCIe
    than the reference's fp32 tensors) get datasets.py:239-250's Resize / ToTensor /
    Normalize on the device (mauv.staging, bit-exact with PIL + torchvision)."""
    t = t.to(device, non_blocking=True)
    if t.dtype == torch.uint8 and t.is_cuda:
        from .staging import stage_tile_batch
        t = stage_tile_batch(t, optical)
    return t


def _batch_to(batch, device, bathy_patch_type, sss_patch_type):
    inputs = _tile_to(batch["main_image"], device, optical=True)
    labels = batch["label"].long().to(device, non_blocking=True)
    # only the selected patch tensors move to the device (the reference copies all of them)
    pb, ps = batch.get("patch_bathy", {}), batch.get("patch_sss", {})
    bathy = _tile_to(pb[bathy_patch_type] if bathy_patch_type in pb else batch["bathy_image"],
                     device)
    sss = _tile_to(ps[sss_patch_type] if sss_patch_type in ps else batch["sss_image"], device)
    return inputs, labels, bathy, sss


class _NullFile:
    """What a non-writing rank "opens" instead of the CSV file."""

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def write(self, s):
        return len(s)


def _patch_tag(t, kind):
    return t.replace("patch_", "").replace(f"_{kind}", "") if t else "none"


def refresh_centres_on_gpu(model):
    """engine.refresh_centres for a model on a ROCm device (the 16-bit storage centres follow
    the running statistics once per training epoch)."""
    from .engine import refresh_centres
    core = unwrap(model)
    p = next(core.parameters(), None)
    if p is not None and p.is_cuda:
        refresh_centres(core)


def train_multimodal_model(multimodal_model, dataloader, criterion, optimizer, epoch, device,
                           model_type, total_num_epochs, num_mc, sum_writer,
                           bathy_patch_type=None, sss_patch_type=None, csv_path=""):
    """train/multimodal.py:25-202 -> (train_loss, train_accuracy)."""
    from .checkpointing import save_model
    multimodal_model.train()
    device = loop_device(multimodal_model, device)
    refresh_centres_on_gpu(multimodal_model)
    writer = is_writer(multimodal_model)
    csv_path = str(Path(csv_path))
    sss_tag, bathy_tag = _patch_tag(sss_patch_type, "sss"), _patch_tag(bathy_patch_type, "bathy")
    new_file = not os.path.isfile(csv_path)
    try:
        with (open(csv_path, mode="a", newline="") if writer else _NullFile()) as fh:
            w = csv.writer(fh)
            if new_file:
                w.writerow(["Epoch", "Model type", "Loss", "Accuracy", "lr", "kl loss",
                            "cross entropy loss", "SSS Patch Type", "Channel Patch Type"])
            kl_w = kl_weight_for(epoch, total_num_epochs)
            ep = _TrainEpoch(epoch, sum_writer)
            for i, batch in enumerate(dataloader):
                inputs, labels, bathy, sss = _batch_to(batch, device, bathy_patch_type,
                                                       sss_patch_type)
                r = mc_train_step(multimodal_model, (inputs, bathy, sss), labels, criterion,
                                  optimizer, num_mc, dataloader.batch_size, kl_w)
                if r is not None:
                    ep.add(i, r, labels)
            ep.flush()
            total_loss, correct, total, last = ep.total_loss, ep.correct, ep.total, ep.last
            # DistributedMC: the epoch's figures over every rank's batches
            total_loss, correct, total = sum_ranks(multimodal_model, [total_loss, correct, total])
            train_accuracy = correct / total
            train_loss = total_loss / total
            lr = optimizer.param_groups[0]["lr"]
            logging.info(f"Epoch {epoch + 1} complete. Loss: {train_loss:.4f}, "
                         f"Accuracy: {train_accuracy:.4f}, LR: {lr:.6f}")
            w.writerow([epoch, model_type, train_loss, train_accuracy, lr,
                        last["scaled_kl"].item(), last["ce"].item(), sss_tag, bathy_tag])
        if epoch % 5 == 0 and writer:
            save_model(multimodal_model, csv_path,
                       f"{model_type}_bathy_patch{bathy_tag}_sss_patch{sss_tag}")
    except Exception:
        if writer:
            save_model(multimodal_model, csv_path,
                       f"{model_type}_bathy_patch{bathy_tag}_sss_patch{sss_tag}")
        logging.error(f"Error at epoch {epoch}", exc_info=True)
        train_loss, train_accuracy = 0.0, 0.0
    return train_loss, train_accuracy


def _confusion_png(cm, csv_path, model_type, epoch):
    """The reference's confusion-matrix PNG (multimodal.py:322-347) from a count matrix."""
    fig = None
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        from sklearn.metrics import ConfusionMatrixDisplay
        fig, ax = plt.subplots(figsize=(8, 8))
        ConfusionMatrixDisplay(confusion_matrix=cm).plot(cmap="Blues", ax=ax)
        plt.title(f"Confusion Matrix for Epoch {epoch}")
        folder = os.path.join(os.path.dirname(csv_path), "confusion_matrices")
        os.makedirs(folder, exist_ok=True)
        plt.savefig(os.path.join(folder, f"conf_matrix_model_{model_type}_{epoch}.png"))
    except Exception as e:
        logging.warning(f"Confusion matrix not saved due to plotting error: {e}")
    finally:
        if fig is not None:
            import matplotlib.pyplot as plt
            plt.close(fig)


class _EvalEpoch:
    """Per-epoch evaluation state with no per-batch device -> host copies: losses, correct
    counts and uncertainties stay on the device (one copy each at the end, summed in the
    reference's order), the confusion counts accumulate in mauv.metrics (metrics.hip).  A
    foreign model's host tensors take the reference's host lists and sklearn."""

    def __init__(self, C):
        self.C, self.acc = C, None
        self.losses, self.correct, self.vals = [], [], {}
        self.labels, self.preds = [], []
        self.total = 0

    def add(self, loss, labels, predicted, **vals):
        self.losses.append(loss.detach().reshape(()))
        self.correct.append((predicted == labels).sum())
        self.total += labels.size(0)
        for k, v in vals.items():
            self.vals.setdefault(k, []).append(v.detach().float().reshape(-1))
        if labels.is_cuda:
            if self.acc is None:
                from .metrics import EvalAccumulator
                self.acc = EvalAccumulator(self.C, labels.device)
            self.acc.update(labels, predicted)
        else:
            self.labels.append(labels)
            self.preds.append(predicted)

    def loss_sum(self):
        return sum(float(v) for v in torch.stack(self.losses).cpu().tolist())

    def correct_count(self):
        return int(torch.stack(self.correct).sum().item())

    def values(self, k):
        """float32 numpy vector of the epoch (the reference's list of np.float32)."""
        return torch.cat(self.vals[k]).cpu().numpy() if k in self.vals else np.zeros(0, np.float32)

    def confusion(self):
        if self.acc is not None:
            return self.acc.confusion_matrix()
        from sklearn.metrics import confusion_matrix
        return confusion_matrix(torch.cat(self.labels).numpy(), torch.cat(self.preds).numpy())


def evaluate_multimodal_model(multimodal_model, dataloader, device, epoch, total_num_epochs,
                              num_mc, model_type, bathy_patch_type=None, sss_patch_type=None,
                              csv_path=""):
    """train/multimodal.py:204-369 -> test accuracy (BN stays in train mode, :232).
    DistributedMC: accuracy, loss and the uncertainty means are taken over every rank's
    batches; rank 0 writes the row and the confusion plot."""
    multimodal_model.train()
    device = loop_device(multimodal_model, device)
    writer = is_writer(multimodal_model)
    csv_path = str(Path(csv_path))
    new_file = not os.path.isfile(csv_path)
    try:
        with (open(csv_path, mode="a", newline="") if writer else _NullFile()) as fh:
            w = csv.writer(fh)
            if new_file:
                w.writerow(["Epoch", "Model Type", "Test Loss", "Test Accuracy",
                            "Predictive Uncertainty", "Model Uncertainty", "Scaled KL",
                            "Cross Entropy Loss", "bathy Patch Type", "SSS Patch Type"])
            kl_w = kl_weight_for(epoch, total_num_epochs)
            ep = None
            with torch.no_grad():
                for batch in dataloader:
                    inputs, labels, bathy, sss = _batch_to(batch, device, bathy_patch_type,
                                                           sss_patch_type)
                    logits = mc_logits(multimodal_model, num_mc, inputs, bathy, sss)
                    kl = get_kl_loss(multimodal_model)
                    kl_scaled = kl / len(dataloader) * kl_w
                    ce, predicted, st = mc_eval_stats(logits, labels, 1e-8, 1e-8)
                    ep = ep or _EvalEpoch(logits.shape[2])
                    pu = st["predictive_entropy"]
                    ep.add(ce + kl_scaled, labels, predicted, pu=pu, mu=pu - st["aleatoric"])
            pu, mu = ep.values("pu"), ep.values("mu")
            correct, total, loss_sum, nb, pu_s, mu_s, n_u = sum_ranks(
                multimodal_model, [ep.correct_count(), ep.total, ep.loss_sum(), len(dataloader),
                                   float(np.sum(pu, dtype=np.float64)),
                                   float(np.sum(mu, dtype=np.float64)), pu.size])
            test_accuracy = correct / total
            test_loss = loss_sum / nb
            if nb == len(dataloader):   # one process: the reference's float32 means
                pu_m, mu_m = np.mean(pu), np.mean(mu)
            else:
                pu_m, mu_m = pu_s / n_u, mu_s / n_u
            if writer:
                _confusion_png(ep.confusion(), csv_path, model_type, epoch)
            w.writerow([epoch + 1, model_type, test_loss, test_accuracy, pu_m,
                        mu_m, kl_scaled.item(), ce.item(),
                        bathy_patch_type or "patch_30_bathy", sss_patch_type or "patch_30_sss"])
            logging.info(f"Epoch {epoch + 1}: Test Loss: {test_loss:.4f}, "
                         f"Accuracy: {test_accuracy:.4f}")
    except Exception as e:
        logging.error(f"Critical error at epoch {epoch}: {e}", exc_info=True)
        test_accuracy = 0.0
    return test_accuracy


_UNI_SOURCES = {"image": "main_image", "sss": "sss_image", "bathy": "bathy_image"}


def train_unimodal_model(model, dataloader, criterion, optimizer, epoch, total_num_epochs,
                         num_mc, sum_writer, device, model_type="image", csv_path="",
                         patch_type=None):
    """train/unimodal.py:21-175 -> (train_accuracy, train_loss) (note the reference's order)."""
    from .checkpointing import save_model
    model.train()
    device = loop_device(model, device)
    model.to(device)
    refresh_centres_on_gpu(model)
    kl_w = kl_weight_for(epoch, total_num_epochs)
    new_file = not os.path.isfile(csv_path)
    try:
        with open(csv_path, mode="a", newline="") as fh:
            w = csv.writer(fh)
            if new_file:
                w.writerow(["Epoch", "Model type", "Loss", "Accuracy", "lr"])
            total_loss, correct, total = 0.0, 0, 0
            for i, batch in enumerate(dataloader):
                if model_type not in _UNI_SOURCES:
                    logging.error(f"Unknown model_type: {model_type}")
                    raise ValueError(f"Unknown model_type: {model_type}")
                x = batch[_UNI_SOURCES[model_type]].to(device, non_blocking=True)
                labels = batch["label"].long().to(device, non_blocking=True)
                optimizer.zero_grad()
                logits = mc_logits(model, num_mc, x)
                kl = get_kl_loss(model)
                if _is_plain_ce(criterion) and logits.is_cuda:
                    ce, output, predicted = mchead.mc_mean_ce(logits, labels)
                else:
                    output = mchead.mc_mean(logits) if logits.is_cuda else logits.mean(0)
                    ce = criterion(output, labels)
                    predicted = output.detach().float().max(1)[1]
                loss = ce + kl_w * (kl / dataloader.batch_size)
                loss.backward()
                optimizer.step()
                lv = loss.item()
                total_loss += lv
                correct += int((predicted == labels).sum().item())
                total += labels.size(0)
                sum_writer.add_scalar("Loss/train", lv, i)
            train_accuracy = correct / total
            train_loss = total_loss / total
            lr = optimizer.param_groups[0]["lr"]
            w.writerow([epoch + 1, model_type, train_loss, train_accuracy, lr])
        if epoch % 5 == 0:
            save_model(model, csv_path, model_type)
    except Exception:
        save_model(model, csv_path, model_type)
        logging.error(f"Error at epoch {epoch}", exc_info=True)
        train_accuracy, train_loss = 0.0, 0.0
    return train_accuracy, train_loss


def evaluate_unimodal_model(model, dataloader, device, epoch, csv_path, total_num_epochs, num_mc,
                            model_type="image", patch_type=None):
    """train/unimodal.py:178-365 -> accuracy (epistemic = var over MC, eps 1e-7 entropy)."""
    model.train()
    device = loop_device(model, device)
    kl_w = kl_weight_for(epoch, total_num_epochs)
    new_file = not os.path.isfile(csv_path)
    try:
        with open(csv_path, mode="a", newline="") as fh:
            w = csv.writer(fh)
            if new_file:
                w.writerow(["Epoch", "Model Type", "Test Loss", "Test Accuracy",
                            "predictive_uncertainty", "model_uncertainty"])
            ep = None
            with torch.no_grad():
                for batch in dataloader:
                    if model_type not in _UNI_SOURCES:
                        raise ValueError(f"Unknown model_type: {model_type}")
                    x = batch[_UNI_SOURCES[model_type]].to(device, non_blocking=True)
                    labels = batch["label"].long().to(device, non_blocking=True)
                    logits = mc_logits(model, num_mc, x)
                    kl = get_kl_loss(model)
                    ce, predicted, st = mc_eval_stats(logits, labels, 1e-7, 1e-7)
                    ep = ep or _EvalEpoch(logits.shape[2])
                    ep.add(ce + kl_w * (kl / dataloader.batch_size), labels, predicted,
                           ep_=st["var"], al=st["aleatoric"])
            accuracy = ep.correct_count() / ep.total
            avg_loss = ep.loss_sum() / ep.total
            all_ep, all_al = ep.values("ep_"), ep.values("al")
            _confusion_png(ep.confusion(), csv_path, model_type, epoch)
            w.writerow([epoch + 1, model_type, avg_loss, accuracy,
                        np.mean(all_ep) if all_ep.size else 0.0,
                        np.mean(all_al) if all_al.size else 0.0])
    except Exception:
        from .checkpointing import save_model
        save_model(model, csv_path, model_type)
        logging.error(f"Error at epoch {epoch}", exc_info=True)
        accuracy = 0.0
    return accuracy
