"""Host logic of the block-output fold (no GPU): which next-block convs the engine folds
(engine.TrunkRunner._fold_fits: 1x1 / stride 1 / no padding, and at least FOLD_MIN_TILES
256-row tiles in the launch), and the argument checks of ops.conv2d_fwd_fold before anything
reaches the library (16-bit weights only; device tensors only — a host pointer reaching a HIP
kernel is a fault the caller cannot catch).  The kernel itself: tests/test_fold_gpu.py."""
import types

import pytest
import torch


def _conv(cin, cout, k, stride, pad, int_kernel=True):
    # bayesian-torch keeps kernel_size an int, torch.nn.Conv2d a tuple: both forms
    return types.SimpleNamespace(in_channels=cin, out_channels=cout,
                                 kernel_size=k if int_kernel else (k, k),
                                 stride=(stride, stride), padding=(pad, pad))


def _runner(G):
    from mauv import engine
    r = engine.TrunkRunner.__new__(engine.TrunkRunner)
    r.G = G
    return r


@pytest.mark.parametrize("int_kernel", [True, False])
def test_fold_fits_shapes_and_tile_rule(int_kernel, monkeypatch):
    from mauv import engine
    monkeypatch.setattr(engine, "FOLD_MIN_TILES", 512)
    r = _runner(5)
    # layer-1 conv1 at the bench's training slice: 64 x 64 x 64 px rows / 256 = 1024 tiles x 5
    assert r._fold_fits(_conv(256, 64, 1, 1, 0, int_kernel), 64, 64, 64)
    # a 3x3 or a strided conv never folds
    assert not r._fold_fits(_conv(256, 64, 3, 1, 1, int_kernel), 64, 64, 64)
    assert not r._fold_fits(_conv(256, 64, 1, 2, 0, int_kernel), 64, 64, 64)
    # layer 4 at B = 64: 64 x 8 x 8 rows -> 16 row tiles x 5 groups x 2 column tiles = 160
    assert not r._fold_fits(_conv(2048, 512, 1, 1, 0, int_kernel), 64, 8, 8)
    # ... folds once the launch has enough tiles (the f16 inference chunk: G = 50, B = 256)
    assert _runner(50)._fold_fits(_conv(2048, 512, 1, 1, 0, int_kernel), 256, 8, 8)
    monkeypatch.setattr(engine, "FOLD_MIN_TILES", 0)
    assert r._fold_fits(_conv(2048, 512, 1, 1, 0, int_kernel), 64, 8, 8)


def test_fold_tile_count_matches_kernel_tiles(monkeypatch):
    """The engine counts 256-row tiles x column tiles of 256 (N >= 256) or 128 columns — the
    kernel's 64-wide tiles for N = 64 are one column tile either way."""
    from mauv import engine
    r = _runner(1)
    for N, cols in ((64, 1), (128, 1), (256, 1), (384, 2), (512, 2)):
        rows = 256 * 7
        monkeypatch.setattr(engine, "FOLD_MIN_TILES", 7 * cols)
        assert r._fold_fits(_conv(512, N, 1, 1, 0), 1, 1, rows)
        monkeypatch.setattr(engine, "FOLD_MIN_TILES", 7 * cols + 1)
        assert not r._fold_fits(_conv(512, N, 1, 1, 0), 1, 1, rows)


def test_conv2d_fwd_fold_argument_checks():
    from mauv import ops
    G, B, H, W, Cin, Cout = 1, 1, 4, 4, 64, 64
    y = torch.zeros(G, B, H, W, Cin, dtype=torch.float16)
    sc = torch.ones(G, Cin)
    w32 = torch.zeros(G, Cout, 1, 1, Cin)
    out = torch.empty_like(y)
    y1 = torch.empty(G, B, H, W, Cout, dtype=torch.float16)
    with pytest.raises(ValueError, match="16-bit"):
        ops.conv2d_fwd_fold(y, sc, sc, y, None, out, w32, y1, G, B, H, W, Cin, Cout)
    w16 = w32.half()
    with pytest.raises(ValueError, match="contiguous"):     # host tensors never reach a kernel
        ops.conv2d_fwd_fold(y, sc, sc, y, None, out, w16, y1, G, B, H, W, Cin, Cout)
