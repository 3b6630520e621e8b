"""Shared recipe for the golden fixtures (seeds, synthetic batches, epsilon stream, digests).

Used both by ``make_golden.py`` (which drives the reference's own code) and by the CPU
tests that re-run the oracle on the same recipe.
"""
import numpy as np
import torch

SEED_MODEL = 0      # torch.manual_seed before define_models (synthetic weights)
SEED_EPS = 1234     # epsilon generator seed (consumed in forward order)
SEED_DATA = 4321    # synthetic batch seed


def make_batches(seed, n_batches, B, S_opt, S_son, num_classes=7):
    """Synthetic triplet batches in the reference's train-dict contract (datasets.py:343-398):
    optical ~ N(0,1) (post-Normalize), bathy ~ U[0,1) with channel 2 = 0
    (image_processing.py:62-65), SSS ~ U[0,1) (ToTensor range), labels uniform."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n_batches):
        bathy = torch.rand(B, 3, S_son, S_son, generator=g)
        bathy[:, 2] = 0
        out.append({
            "main_image": torch.randn(B, 3, S_opt, S_opt, generator=g),
            "bathy_image": bathy,
            "sss_image": torch.rand(B, 1, S_son, S_son, generator=g),
            "label": torch.randint(0, num_classes, (B,), generator=g),
            "patch_bathy": {},
            "patch_sss": {},
        })
    return out


def eps_generator_source(seed):
    g = torch.Generator().manual_seed(seed)

    def src(layer, name, shape):
        return torch.randn(shape, generator=g)
    return src


class RecordingEpsSource:
    """Epsilon source that also records each draw keyed by (layer object, name)."""

    def __init__(self, seed):
        self.g = torch.Generator().manual_seed(seed)
        self.log = []

    def __call__(self, layer, name, shape):
        e = torch.randn(shape, generator=self.g)
        self.log.append((layer, name, e))
        return e


def param_digest(model):
    tot = np.float64(0)
    tot_abs = np.float64(0)
    tot_sq = np.float64(0)
    n = 0
    for p in model.parameters():
        a = p.detach().double()
        tot += float(a.sum())
        tot_abs += float(a.abs().sum())
        tot_sq += float((a * a).sum())
        n += a.numel()
    return {"n": n, "sum": float(tot), "abs": float(tot_abs), "sq": float(tot_sq)}
