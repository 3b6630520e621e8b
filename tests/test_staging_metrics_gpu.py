"""Device input staging (staging.hip) and evaluation metrics (metrics.hip) — SURVEY.md §8f
rows 2 and 4 — against the oracle / the libraries the reference calls.

Staging: ToTensor + Normalize bit-exact with torchvision's fp32 ops (oracle/staging_ref.py);
the UIFM degradation against the reference's own function's outputs (golden_staging.npz):
exp may differ by one ulp between libm implementations, so |d| <= 5e-7 (outputs in [0, 1],
inputs up to |4|).  Metrics: confusion matrix and AUROC exact (integer counts), macro F1 and
ECE / Emax within 1e-6 of sklearn / the noise script's calibration_metrics (float32 numpy
means there, float64 sums here)."""
import os

import numpy as np
import pytest
import torch

from oracle import staging_ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("B,H,W,C,norm", [(3, 17, 13, 3, True), (2, 256, 256, 3, True),
                                          (2, 31, 40, 1, False), (0, 8, 8, 3, True)])
def test_stage_u8_bit_exact(B, H, W, C, norm):
    from mauv.staging import to_tensor_normalize, OPTICAL_MEAN, OPTICAL_STD
    g = torch.Generator().manual_seed(B * 1000 + H + W + C)
    tiles = torch.randint(0, 256, (B, H, W, C), generator=g, dtype=torch.uint8)
    mean, std = (OPTICAL_MEAN, OPTICAL_STD) if norm and C == 3 else (None, None)
    got = to_tensor_normalize(tiles.to(DEV), mean, std)
    ref = staging_ref.to_tensor_normalize(tiles, mean, std)
    assert got.shape == ref.shape
    assert torch.equal(got.cpu(), ref)


def test_uifm_matches_reference_golden():
    from mauv.staging import simulate_underwater_degradation as sim
    S = np.load(os.path.join(HERE, "golden_staging.npz"))
    clean, dmap = torch.from_numpy(S["clean"]).to(DEV), torch.from_numpy(S["dmap"]).to(DEV)
    ones = torch.ones_like(dmap)
    for i, (turb, depth) in enumerate(((0.3, 1), (1.5, 1), (0.9, 2.5))):
        for m, key in ((ones, "uniform"), (dmap, "map")):
            got = sim(clean, m, turb, depth).cpu().numpy()
            np.testing.assert_allclose(got, S[f"{key}_{i}"], rtol=0, atol=5e-7)


def test_stage_u8_fused_degradation():
    """Normalise + UIFM in one pass == the oracle's normalise, then degrade."""
    from mauv.staging import to_tensor_normalize, OPTICAL_MEAN, OPTICAL_STD
    g = torch.Generator().manual_seed(5)
    tiles = torch.randint(0, 256, (4, 64, 64, 3), generator=g, dtype=torch.uint8)
    dmap = torch.rand(4, 1, 64, 64, generator=g) * 2
    for dist in (None, dmap):
        got = to_tensor_normalize(tiles.to(DEV), OPTICAL_MEAN, OPTICAL_STD,
                                  degrade=(0.7, 1.0) if dist is None else (0.7, 1.0, dist.to(DEV)))
        x = staging_ref.to_tensor_normalize(tiles, OPTICAL_MEAN, OPTICAL_STD)
        ref = staging_ref.simulate_underwater_degradation(
            x, torch.ones(4, 1, 64, 64) if dist is None else dist, 0.7, 1.0)
        np.testing.assert_allclose(got.cpu().numpy(), ref.numpy(), rtol=0, atol=5e-7)


def _calibration_ref(probabilities, labels, n_bins=15):
    """Examples/"Example training with image noise.py":548-563, verbatim maths."""
    confidences = np.max(probabilities, axis=1)
    predictions = np.argmax(probabilities, axis=1)
    accuracies = predictions == labels
    bin_boundaries = np.linspace(0, 1, n_bins + 1)
    ece, emax = 0.0, 0.0
    for i in range(n_bins):
        in_bin = (confidences > bin_boundaries[i]) & (confidences <= bin_boundaries[i + 1])
        prop_in_bin = np.mean(in_bin)
        if prop_in_bin > 0:
            acc_in_bin = np.mean(accuracies[in_bin])
            conf_in_bin = np.mean(confidences[in_bin])
            ece += np.abs(acc_in_bin - conf_in_bin) * prop_in_bin
            emax = max(emax, np.abs(acc_in_bin - conf_in_bin))
    return ece, emax


@pytest.mark.parametrize("n,C,batches", [(1000, 7, 4), (37, 7, 3), (5000, 3, 2)])
def test_eval_metrics_match_sklearn(n, C, batches):
    from sklearn.metrics import confusion_matrix, f1_score, roc_auc_score
    from mauv.metrics import EvalAccumulator
    g = torch.Generator().manual_seed(n + C)
    labels = torch.randint(0, C, (n,), generator=g)
    logits = torch.randn(n, C, generator=g) * 2
    logits[torch.arange(n), labels] += 1.0          # better than chance
    probs = torch.softmax(logits, 1)
    pred = probs.argmax(1)
    unc = torch.rand(n, generator=g)
    unc[: n // 10] = 0.5                             # ties in the AUROC scores
    if C == 3:
        pred[pred == 2] = 1                          # a class absent from the predictions
    acc = EvalAccumulator(C, DEV)
    for idx in torch.arange(n).chunk(batches):
        acc.update(labels[idx].to(DEV), pred[idx].to(DEV), probs[idx].to(DEV), unc[idx].to(DEV))
    y, p = labels.numpy(), pred.numpy()
    np.testing.assert_array_equal(acc.confusion_matrix(), confusion_matrix(y, p))
    assert abs(acc.f1_macro() - f1_score(y, p, average="macro")) <= 1e-12
    ece, emax = acc.calibration()
    ece_r, emax_r = _calibration_ref(probs.numpy(), y)
    assert abs(ece - ece_r) <= 1e-6 and abs(emax - emax_r) <= 1e-6
    auroc = acc.uncertainty_error_auroc()
    assert abs(auroc - roc_auc_score((p != y).astype(int), unc.numpy())) <= 1e-12
    assert acc.accuracy() == float((p == y).mean())


def test_eval_metrics_edge_cases():
    from mauv.metrics import EvalAccumulator
    acc = EvalAccumulator(7, DEV)
    y = torch.tensor([1, 1, 3], device=DEV)
    acc.update(y, y.clone(), uncertainty=torch.rand(3, device=DEV))
    assert acc.confusion_matrix().tolist() == [[2, 0], [0, 1]]
    with pytest.raises(ValueError, match="Only one class"):
        acc.uncertainty_error_auroc()        # every prediction right: one class only
    bad = EvalAccumulator(3, DEV)
    bad.update(torch.tensor([0, 5], device=DEV), torch.tensor([0, 1], device=DEV))
    with pytest.raises(ValueError, match="outside"):
        bad.confusion_matrix()
