"""Device Resize: data/datasets.py:240-246 applies
``transforms.Resize((256, 256))`` to every decoded PIL tile before ToTensor / Normalize, i.e.
PIL's Image.resize(size, BILINEAR).  The oracle (oracle/staging_ref.py) restates Pillow's 8-bit
resampler and is pinned bit-exact to Pillow itself (the committed fixture of
tests/golden/make_resize_golden.py, and live Pillow where importable); the HIP path
(mauv.staging.resize / resize_to_tensor) is held bit-exact to both."""
import os

import numpy as np
import pytest
import torch

from oracle import staging_ref

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "resize_golden.npz")


def _cases():
    d = np.load(GOLD)
    return [(d[f"in{i}"], d[f"out{i}"]) for i in range(len([k for k in d.files if k[:2] == "in"]))]


def test_oracle_resize_matches_pillow_fixture():
    for a, ref in _cases():
        o = staging_ref.pil_resize_bilinear(a, ref.shape[0], ref.shape[1])
        assert o.dtype == np.uint8 and np.array_equal(o, ref), a.shape


def test_oracle_resize_matches_live_pillow():
    pytest.importorskip("PIL")
    from tests.golden.make_resize_golden import pil_resize
    rng = np.random.default_rng(5)
    for H, W, C in ((300, 420, 3), (256, 256, 3), (150, 900, 1)):
        a = rng.integers(0, 256, (H, W, C), dtype=np.uint8)
        assert np.array_equal(staging_ref.pil_resize_bilinear(a, 256, 256), pil_resize(a, 256, 256))


@pytest.mark.gpu
def test_device_resize_bit_exact():
    from mauv import staging
    for a, ref in _cases():
        x = torch.from_numpy(np.stack([a, a[::-1].copy()])).cuda()       # B = 2
        out = staging.resize(x, (ref.shape[0], ref.shape[1])).cpu().numpy()
        assert np.array_equal(out[0], ref), a.shape
        assert np.array_equal(out[1], staging_ref.pil_resize_bilinear(a[::-1].copy(), *ref.shape[:2]))
    rng = np.random.default_rng(6)
    for H, W, C in ((300, 420, 3), (513, 1000, 3), (256, 256, 1), (64, 80, 1)):
        a = rng.integers(0, 256, (3, H, W, C), dtype=np.uint8)
        out = staging.resize(torch.from_numpy(a).cuda(), 256).cpu().numpy()
        for b in range(3):
            assert np.array_equal(out[b], staging_ref.pil_resize_bilinear(a[b], 256, 256)), (H, W, C)


@pytest.mark.gpu
def test_device_resize_to_tensor_normalize_and_degrade():
    """Compose([Resize((256, 256)), ToTensor(), Normalize(mean, std)]) fused in one pass,
    bit-exact with the oracle's torch fp32 ops on the Pillow-resized tile; with the UIFM
    degradation of the noise scripts on top."""
    from mauv import staging
    rng = np.random.default_rng(7)
    a = rng.integers(0, 256, (2, 300, 420, 3), dtype=np.uint8)
    x = torch.from_numpy(a).cuda()
    rs = np.stack([staging_ref.pil_resize_bilinear(t, 256, 256) for t in a])
    ref = staging_ref.to_tensor_normalize(torch.from_numpy(rs), staging.OPTICAL_MEAN,
                                          staging.OPTICAL_STD)
    out = staging.resize_to_tensor(x, (256, 256), staging.OPTICAL_MEAN, staging.OPTICAL_STD)
    assert torch.equal(out.cpu(), ref)
    plain = staging.resize_to_tensor(x, (256, 256))                     # ToTensor only
    assert torch.equal(plain.cpu(), staging_ref.to_tensor_normalize(torch.from_numpy(rs)))
    deg = staging.resize_to_tensor(x, (256, 256), degrade=(1.5, 0.7))
    ref_d = staging_ref.simulate_underwater_degradation(
        staging_ref.to_tensor_normalize(torch.from_numpy(rs)), torch.ones(2, 1, 256, 256), 1.5,
        0.7)
    assert (deg.cpu() - ref_d).abs().max().item() <= 1e-6


@pytest.mark.gpu
def test_dropin_loops_stage_uint8_tiles(tmp_path):
    """The drop-in loops take decoded uint8 HWC tiles and run datasets.py:239-250's transforms
    on the device: the staged batch equals the reference's host-transformed fp32 batch, and the
    predictor writes the same CSV from either."""
    import csv
    from mauv.train import _batch_to
    from mauv.predict import multimodal_predict_and_save
    from mauv.engine import root_state
    from mauv import staging
    from tests.helpers import build_pair
    rng = np.random.default_rng(8)
    B = 3
    opt8 = rng.integers(0, 256, (B, 300, 420, 3), dtype=np.uint8)
    bat8 = rng.integers(0, 256, (B, 200, 180, 3), dtype=np.uint8)
    sss8 = rng.integers(0, 256, (B, 90, 600, 1), dtype=np.uint8)

    def host(a, norm):   # the reference: PIL Resize + ToTensor (+ Normalize) on CPU workers
        rs = torch.from_numpy(np.stack([staging_ref.pil_resize_bilinear(t, 256, 256) for t in a]))
        return staging_ref.to_tensor_normalize(
            rs, *((staging.OPTICAL_MEAN, staging.OPTICAL_STD) if norm else (None, None)))
    ref = {"main_image": host(opt8, True), "bathy_image": host(bat8, False),
           "sss_image": host(sss8, False), "label": torch.tensor([1, 2, 3])}
    raw = {"main_image": torch.from_numpy(opt8), "bathy_image": torch.from_numpy(bat8),
           "sss_image": torch.from_numpy(sss8), "label": torch.tensor([1, 2, 3])}
    got, want = _batch_to(raw, "cuda", None, None), _batch_to(ref, "cuda", None, None)
    for g, w in zip(got, want):
        assert g.dtype == w.dtype and torch.equal(g, w)
    _, m = build_pair()
    rows = []
    for bt in (raw, ref):
        root_state(m).offset = 0
        p = tmp_path / f"p{len(rows)}.csv"
        multimodal_predict_and_save(m, [(bt["main_image"], bt["bathy_image"], bt["sss_image"],
                                         ["a", "b", "c"])], "cuda", str(p), num_mc_samples=3)
        rows.append(list(csv.reader(open(p))))
    assert rows[0] == rows[1]
