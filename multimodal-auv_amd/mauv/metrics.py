"""Evaluation metrics accumulated on the device (metrics.hip).

The reference copies each eval batch's predictions, labels and uncertainties to the host
(train/multimodal.py:312-321) and computes, once per epoch, sklearn's ``confusion_matrix``
(:322-347) and — in the noise scripts (Examples/"Example training with image
noise.py":530-634) — the uncertainty-vs-error ``roc_auc_score``, macro ``f1_score`` and a
15-bin ECE / Emax of the MC-mean softmax.  ``EvalAccumulator`` keeps the per-sample work on
the GPU across the epoch (confusion counts, calibration bins, the AUROC pair count) and
hands the host a C x C matrix and a few scalars.  Semantics follow sklearn / the reference:

* ``confusion_matrix()``  rows true, columns predicted, restricted to the classes present in
  labels or predictions (sklearn's default ``labels``), int64;
* ``f1_macro()``          per present class 2TP / (2TP + FP + FN) (0 where undefined, sklearn's
  zero_division default), averaged;
* ``calibration(n_bins)`` (ECE, Emax) with bins (b_i, b_i+1] on ``np.linspace(0, 1, n+1)``;
* ``uncertainty_error_auroc()``  AUROC of the uncertainty as a score for "prediction wrong";
  ValueError when only one of the two classes occurs (as roc_auc_score).
"""
import numpy as np
import torch

from . import ops
from ._lib import lib, check


class EvalAccumulator:
    def __init__(self, num_classes, device, n_bins=15):
        self.C, self.dev, self.n_bins = int(num_classes), torch.device(device), n_bins
        self.counts = torch.zeros(self.C * self.C + 1, dtype=torch.int32, device=self.dev)
        self.edges = torch.tensor(np.linspace(0, 1, n_bins + 1), dtype=torch.float64,
                                  device=self.dev)
        self.bins = torch.zeros(n_bins, 3, dtype=torch.float64, device=self.dev)
        self.n = 0
        self._scores, self._wrong = [], []

    def update(self, labels, predicted, mean_prob=None, uncertainty=None):
        """One batch: labels / predicted [B] (int64), MC-mean probabilities [B, C] (for the
        calibration), per-sample uncertainty [B] (for the AUROC)."""
        labels = labels.to(self.dev, torch.int64).contiguous()
        predicted = predicted.to(self.dev, torch.int64).contiguous()
        n = labels.numel()
        ops._dev(torch.int64, labels, predicted)
        check(lib.mauv_confusion_update(labels.data_ptr(), predicted.data_ptr(), n, self.C,
                                        self.counts.data_ptr(), ops.stream()), "confusion")
        if mean_prob is not None:
            p = mean_prob.to(self.dev, torch.float32).contiguous()
            if p.shape != (n, self.C):
                raise ValueError(f"mean_prob must be [{n}, {self.C}]")
            check(lib.mauv_calibration_update(p.data_ptr(), labels.data_ptr(), n, self.C,
                                              self.n_bins, self.edges.data_ptr(),
                                              self.bins.data_ptr(), ops.stream()), "calibration")
        if uncertainty is not None:
            self._scores.append(uncertainty.to(self.dev, torch.float32).reshape(-1))
            self._wrong.append((predicted != labels).to(torch.uint8))
        self.n += n

    # ---- epoch results (one small device -> host copy each) ----
    def _counts(self):
        c = self.counts.cpu().numpy().astype(np.int64)
        if c[-1]:
            raise ValueError(f"{c[-1]} labels / predictions outside [0, {self.C})")
        return c[:-1].reshape(self.C, self.C)

    def confusion_matrix(self):
        full = self._counts()
        present = np.nonzero(full.sum(0) + full.sum(1))[0]
        return full[np.ix_(present, present)]

    def accuracy(self):
        full = self._counts()
        return float(np.trace(full)) / max(int(full.sum()), 1)

    def f1_macro(self):
        cm = self.confusion_matrix()
        tp = np.diag(cm).astype(np.float64)
        fp = cm.sum(0) - tp
        fn = cm.sum(1) - tp
        den = 2 * tp + fp + fn
        f1 = np.where(den > 0, 2 * tp / np.where(den > 0, den, 1), 0.0)
        return float(f1.mean()) if f1.size else 0.0

    def calibration(self):
        """(ECE, Emax) of the MC-mean softmax (noise script calibration_metrics)."""
        b = self.bins.cpu().numpy()
        ece, emax = 0.0, 0.0
        for cnt, sconf, sacc in b:
            if cnt > 0:
                gap = abs(sacc / cnt - sconf / cnt)
                ece += gap * (cnt / self.n)
                emax = max(emax, gap)
        return ece, emax

    def uncertainty_error_auroc(self):
        if not self._scores:
            raise ValueError("no uncertainties accumulated")
        s = torch.cat(self._scores).contiguous()
        w = torch.cat(self._wrong).contiguous()
        n_pos = int(w.sum().item())
        n_neg = w.numel() - n_pos
        if n_pos == 0 or n_neg == 0:
            raise ValueError("Only one class present in y_true. ROC AUC score is not defined "
                             "in that case.")
        cnt = torch.zeros(1, dtype=torch.int64, device=self.dev)
        check(lib.mauv_auroc_pairs(s.data_ptr(), w.data_ptr(), s.numel(), cnt.data_ptr(),
                                   ops.stream()), "auroc")
        return int(cnt.item()) / (2.0 * n_pos * n_neg)
