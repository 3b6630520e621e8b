"""Oracle: per-batch maths of the reference's MC loops (TEST INFRASTRUCTURE ONLY).

* ``train_step_multimodal``  train/multimodal.py:80-155 (sequential MC loop :107-118, mean of
  logits :121, KL mean / dataloader.batch_size * kl_weight :124, CE :127, NaN/Inf skip :133,
  backward :138, grad NaN/Inf guard :141-145 — zero_grad only after a successful step)
* ``eval_batch_multimodal``  train/multimodal.py:276-310 (H[p_bar] eps 1e-8 :305-306,
  E_N H[p] :308-309, epistemic = difference :310, KL / len(dataloader) :293)
* ``predict_batch``          inference/predictors.py:54-84 (softmax per pass :65, unbiased var
  over MC then mean over classes :73, aleatoric with eps 1e-7 :77-79, argmax of mean prob :83)
* ``train_step_unimodal``    train/unimodal.py:110-146 (zero_grad first :110, MC :127-130,
  loss = CE + kl_weight * mean(KL)/batch_size :136-142)
"""
import torch
import torch.nn.functional as F

from .bayes_ref import get_kl_loss


def kl_weight(epoch, total_num_epochs):
    return (2 ** (epoch + 1)) / (2 ** total_num_epochs)  # multimodal.py:80, unimodal.py:71


def mc_logits(model, inputs, bathy, sss, num_mc):
    return torch.stack([model(inputs, bathy, sss) for _ in range(num_mc)])


def train_step_multimodal(model, inputs, bathy, sss, labels, criterion, optimizer, epoch,
                          total_num_epochs, num_mc, batch_size):
    kw = kl_weight(epoch, total_num_epochs)
    outs, kls = [], []
    for _ in range(num_mc):
        outs.append(model(inputs, bathy, sss))
        kls.append(get_kl_loss(model))
    output = torch.mean(torch.stack(outs), dim=0)
    scaled_kl = torch.mean(torch.stack(kls), dim=0) / batch_size * kw
    ce = criterion(output, labels)
    loss = ce + scaled_kl
    if torch.any(torch.isnan(loss)) or torch.any(torch.isinf(loss)):
        return dict(skipped=True, loss=loss.detach(), output=output.detach())
    loss.backward()
    stepped = False
    if not any(torch.any(torch.isnan(p.grad)) or torch.any(torch.isinf(p.grad))
               for p in model.parameters() if p.grad is not None):
        optimizer.step()
        optimizer.zero_grad()
        stepped = True
    _, predicted = torch.max(output, 1)
    return dict(skipped=False, stepped=stepped, loss=loss.detach(), ce=ce.detach(),
                scaled_kl=scaled_kl.detach(), output=output.detach(), predicted=predicted,
                correct=int((predicted == labels).sum()))


def eval_batch_multimodal(model, inputs, bathy, sss, labels, epoch, total_num_epochs, num_mc,
                          num_batches):
    kw = kl_weight(epoch, total_num_epochs)
    eps = 1e-8
    with torch.no_grad():
        outs, probs, kls = [], [], []
        for _ in range(num_mc):
            o = model(inputs, bathy, sss)
            outs.append(o)
            probs.append(F.softmax(o, dim=1))
            kls.append(get_kl_loss(model))
        out_mean = torch.mean(torch.stack(outs), dim=0)
        P = torch.stack(probs)
        kl_scaled = torch.mean(torch.stack(kls), dim=0) / num_batches * kw
        ce = F.cross_entropy(out_mean, labels)
        loss = ce + kl_scaled
        _, predicted = torch.max(out_mean, 1)
        mean_p = P.mean(0)
        pred_unc = -torch.sum(mean_p * torch.log(mean_p + eps), dim=1)
        alea = torch.mean(-torch.sum(P * torch.log(P + eps), dim=2), dim=0)
        return dict(loss=loss, ce=ce, kl_scaled=kl_scaled, predicted=predicted,
                    predictive_uncertainty=pred_unc, model_uncertainty=pred_unc - alea,
                    correct=int((predicted == labels).sum()), logits=torch.stack(outs))


def mc_uncertainty_from_probs(P):
    """predictors.py:73-84 applied to a stacked [N, B, C] probability tensor."""
    predictive = torch.var(P, dim=0).mean(dim=1)
    alea = torch.mean(-torch.sum(P * torch.log(P + 1e-7), dim=-1), dim=0)
    pred = torch.argmax(torch.mean(P, dim=0), dim=1)
    return pred, predictive, alea


def predict_batch(model, inputs, bathy, sss, num_mc, autocast=False):
    with torch.no_grad():
        probs = []
        for _ in range(num_mc):
            with torch.amp.autocast(device_type="cpu", enabled=autocast):
                out = model(inputs, bathy, sss)
                probs.append(F.softmax(out, dim=1))
        P = torch.stack(probs, dim=0)
        return mc_uncertainty_from_probs(P) + (P,)


def train_step_unimodal(model, x, labels, criterion, optimizer, epoch, total_num_epochs,
                        num_mc, batch_size):
    kw = kl_weight(epoch, total_num_epochs)
    optimizer.zero_grad()
    outs, kls = [], []
    for _ in range(num_mc):
        outs.append(model(x))
        kls.append(get_kl_loss(model))
    output = torch.mean(torch.stack(outs), dim=0)
    scaled_kl = torch.mean(torch.stack(kls), dim=0) / batch_size
    ce = criterion(output, labels)
    loss = ce + kw * scaled_kl
    loss.backward()
    optimizer.step()
    _, predicted = output.float().max(1)
    return dict(loss=loss.detach(), output=output.detach(), predicted=predicted,
                correct=int((predicted == labels).sum()))
