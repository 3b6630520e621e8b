"""Fused MC-head reductions as autograd ops (train/multimodal.py:121-127,287-310;
inference/predictors.py:65-84): mean of logits over the MC samples, cross-entropy, argmax and
the uncertainty statistics — one kernel each instead of stack/mean/softmax/log/var chains.
"""
import torch

from . import ops


class _MCMeanCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        G, B, C = logits.shape
        mean = torch.empty(B, C, device=logits.device)
        loss = torch.empty(1, device=logits.device)
        pred = torch.empty(B, dtype=torch.int64, device=logits.device)
        ops.mc_mean_ce(logits, labels, G, B, C, mean, loss, pred)
        ctx.save_for_backward(mean, labels)
        ctx.G = G
        ctx.mark_non_differentiable(mean, pred)
        return loss[0], mean, pred

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gloss, gmean, gpred):
        mean, labels = ctx.saved_tensors
        B, C = mean.shape
        dl = torch.empty(ctx.G, B, C, device=mean.device)
        ops.mc_mean_bwd(None, gloss.reshape(1).float().contiguous(), mean, labels, ctx.G, B, C,
                        dl)
        return dl, None


class _MCMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits):
        G, B, C = logits.shape
        mean = torch.empty(B, C, device=logits.device)
        ops.mc_mean_ce(logits, None, G, B, C, mean, None, None)
        ctx.G = G
        return mean

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gmean):
        B, C = gmean.shape
        dl = torch.empty(ctx.G, B, C, device=gmean.device)
        ops.mc_mean_bwd(gmean.contiguous().float(), None, None, None, ctx.G, B, C, dl)
        return dl


def mc_mean_ce(logits, labels):
    """-> (cross-entropy of the MC-mean logits [0-d], mean logits [B,C], argmax [B])."""
    return _MCMeanCE.apply(logits.contiguous(), labels.long().contiguous())


def mc_mean(logits):
    return _MCMean.apply(logits.contiguous())


def mc_stats(logits, eps_h, sums=None):
    """Accumulate sum p, sum p^2, sum H[p] over the MC samples of ``logits`` [G,B,C] into
    ``sums`` [B, 2C+1] float64 (created if None) — shardable across ranks."""
    G, B, C = logits.shape
    acc = sums is not None
    if sums is None:
        sums = torch.empty(B, 2 * C + 1, dtype=torch.float64, device=logits.device)
    ops.mc_stats(logits.contiguous(), G, B, C, eps_h, sums, accumulate=acc)
    return sums


def mc_finalize(sums, N, C, eps_pred):
    """-> dict(mean_prob [B,C], var [B] (unbiased over MC, mean over classes), aleatoric [B],
    predictive_entropy [B], pred [B])."""
    B = sums.shape[0]
    dev = sums.device
    out = dict(mean_prob=torch.empty(B, C, device=dev), var=torch.empty(B, device=dev),
               aleatoric=torch.empty(B, device=dev), predictive_entropy=torch.empty(B, device=dev),
               pred=torch.empty(B, dtype=torch.int64, device=dev))
    ops.mc_finalize(sums, N, B, C, eps_pred, out["mean_prob"], out["var"], out["aleatoric"],
                    out["predictive_entropy"], out["pred"])
    return out


def all_finite(tensors_or_flat):
    """One fused non-finite scan (+ one host sync) instead of a per-tensor isnan/isinf loop."""
    ts = tensors_or_flat if isinstance(tensors_or_flat, (list, tuple)) else [tensors_or_flat]
    cnt = torch.zeros(1, dtype=torch.int32, device=ts[0].device)
    for t in ts:
        ops.nonfinite_count(t.detach().contiguous().float(), cnt)
    return int(cnt.item()) == 0
