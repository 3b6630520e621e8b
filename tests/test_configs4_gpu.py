"""BASELINE configs[4]'s MC-inference leg on one GPU: 100 MC passes over 256 triplets at the
sonar-patch sweep's 128 / 512 px (224 px optical), through the drop-in
``multimodal_predict_and_save`` (inference/predictors.py:9-97; main.py:313-314 patch sizes)
under its own f16 autocast, the multi-chunk path at 512 px.

Size-independent properties (no CPU oracle finishes this size in seconds):
* the CSV holds one well-formed row per image (class in range, 0 <= aleatoric <= log C,
  0 <= variance <= p(1-p) N/(N-1) averaged over classes);
* the f16 trunks agree with the fp32 trunks on the SAME Philox stream (same epsilons, so the
  two differ only by the trunk arithmetic, which the fp32 parity tests pin to the oracle):
  predicted class on >= 99 % of the items of a model trained a few steps (``fit_model``),
  aleatoric within 2e-2 and variance within 2e-3 absolute;
* chunking is exact: the statistics do not depend on the MC chunk size.
"""
import csv
import math

import pytest
import torch

from tests.helpers import build_pair, fit_model

pytestmark = pytest.mark.gpu


def _batch(B, S, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, 3, 224, 224, generator=g)
    bathy = torch.rand(B, 3, S, S, generator=g)
    bathy[:, 2] = 0
    sss = torch.rand(B, 1, S, S, generator=g)
    return [t.cuda() for t in (x, bathy, sss)]


@pytest.mark.parametrize("S", [128, 512])
def test_configs4_mc_inference(S, tmp_path):
    from mauv.engine import root_state
    from mauv.predict import mc_statistics, mc_chunk, multimodal_predict_and_save
    _, m = build_pair()
    B, N, C = 256, 100, 7
    x, b, s = _batch(B, S, 7 + S)
    # a few training steps on 32 of the tiles so that the class depends on the input
    fit_model(m, x[:32], b[:32], s[:32],
              torch.randint(0, C, (32,), generator=torch.Generator().manual_seed(4)).cuda())
    hw = [(224, 224), (S, S), (S, S)]
    chunk16 = mc_chunk(m, B, N, dtype=torch.float16, device=x.device, hw=hw)
    if S == 512:
        assert chunk16 < N      # 512 px takes the accumulate path
    names = [f"tile_{i}" for i in range(B)]
    path = tmp_path / "pred.csv"
    multimodal_predict_and_save(m, [(x, b, s, names)], "cuda", str(path), num_mc_samples=N)
    rows = list(csv.reader(open(path)))
    assert rows[0] == ["Image Name", "Predicted Class", "Predictive Uncertainty",
                       "Aleatoric Uncertainty"] and len(rows) == B + 1
    for i, r in enumerate(rows[1:]):
        assert r[0] == names[i] and 0 <= int(r[1]) < C
        v, a = float(r[2]), float(r[3])
        assert math.isfinite(v) and math.isfinite(a)
        assert v >= 0 and -1e-6 <= a <= math.log(C) + 1e-5

    st_ = root_state(m)
    stats = {}
    for key, amp, chunk in (("f16", True, None), ("f16_chunk7", True, 7), ("fp32", False, None)):
        st_.offset = 0          # the same MC samples (Philox counters) for every run
        with torch.no_grad(), torch.autocast("cuda", enabled=amp):
            stats[key] = {k: v.cpu() for k, v in
                          mc_statistics(m, x, b, s, N, chunk=chunk).items()}
    h, c, f = stats["f16"], stats["f16_chunk7"], stats["fp32"]
    for k in ("mean_prob", "var", "aleatoric", "predictive_entropy", "pred"):
        assert torch.equal(h[k], c[k]), k          # chunking is exact
    mp = h["mean_prob"]
    assert (h["var"] <= (mp * (1 - mp)).mean(1) * N / (N - 1) + 1e-6).all()
    assert (h["predictive_entropy"] - h["aleatoric"] >= -1e-4).all()
    classes = len(set(f["pred"].tolist()))
    agree = (h["pred"] == f["pred"]).float().mean().item()
    da = (h["aleatoric"] - f["aleatoric"]).abs().max().item()
    dv = (h["var"] - f["var"]).abs().max().item()
    print(f"\nS={S}: f16 chunk {chunk16}; {classes} classes; f16 vs fp32 trunks: argmax agreement "
          f"{agree:.4f}, max |dalea| {da:.2e}, max |dvar| {dv:.2e}")
    assert classes >= 3
    assert agree >= 0.99
    assert da <= 2e-2 and dv <= 2e-3
