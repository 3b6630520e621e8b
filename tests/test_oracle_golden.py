"""Pin the oracle against golden vectors produced by the REFERENCE's own code
(tests/golden/make_golden.py drives models/model_utils.py:define_models,
base_models.py:MultiModalModel, train/multimodal.py:train_multimodal_model /
evaluate_multimodal_model, inference/predictors.py:multimodal_predict_and_save and
train/unimodal.py:train_unimodal_model with the oracle's third-party restatements injected).
Here the oracle runs standalone — no reference import — and must reproduce them."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import bayes_ref, loops_ref
from oracle.model_ref import define_models, DEFAULT_PRIOR
from tests.golden.common import (SEED_MODEL, SEED_EPS, SEED_DATA, make_batches,
                                 eps_generator_source, param_digest)

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
G = json.load(open(os.path.join(HERE, "golden.json")))
A = np.load(os.path.join(HERE, "golden.npz"))


@pytest.fixture(autouse=True)
def _threads():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    yield
    bayes_ref.set_eps_source(None)


def _models():
    torch.manual_seed(SEED_MODEL)
    return define_models(None, 7, DEFAULT_PRIOR)


def _digest_close(d, ref, rel=1e-6):
    assert d["n"] == ref["n"]
    for k in ("sum", "abs", "sq"):
        assert abs(d[k] - ref[k]) <= rel * abs(ref[k]) + 1e-6, (k, d[k], ref[k])


def test_known_answers():
    from oracle.resnet_ref import resnet50
    assert sum(p.numel() for p in resnet50().parameters()) == 25_557_032
    m = _models()["multimodal_model"]
    assert sum(p.numel() for p in m.parameters()) == 146_767_638
    assert sum(p.numel() for n, p in m.named_parameters() if ".mu_" in n or n.startswith("mu_")) \
        == 73_304_139
    assert len(list(m.parameters())) == 696


def test_g3_multimodal_forward_matches_reference():
    m = _models()["multimodal_model"]
    b = make_batches(SEED_DATA, 2, B=2, S_opt=64, S_son=64)[0]
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS))
    with torch.no_grad():
        lg = torch.stack([m(b["main_image"], b["bathy_image"], b["sss_image"]) for _ in range(3)])
    np.testing.assert_array_equal(lg.numpy(), A["g3_logits"])
    assert abs(float(bayes_ref.get_kl_loss(m)) - G["g3_kl"]) <= 1e-6 * abs(G["g3_kl"])
    _digest_close(param_digest(m), G["g3_param_digest"])
    np.testing.assert_array_equal(m.image_model_feat.bn1.running_mean.numpy(),
                                  A["g3_bn1_running_mean"])


def test_g5_train_epoch_matches_reference():
    m = _models()["multimodal_model"]
    batches = make_batches(SEED_DATA, 2, B=2, S_opt=64, S_son=64)
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 1))
    opt = torch.optim.Adam(m.parameters(), lr=5e-5)
    crit = torch.nn.CrossEntropyLoss()
    total, correct, n = 0.0, 0, 0
    for b in batches:
        r = loops_ref.train_step_multimodal(m, b["main_image"], b["bathy_image"], b["sss_image"],
                                            b["label"], crit, opt, 0, 2, 2, 2)
        total += float(r["loss"])
        correct += r["correct"]
        n += 2
    assert abs(total / n - G["g5_loss"]) <= 1e-6 * abs(G["g5_loss"])
    assert correct / n == G["g5_acc"]
    row = G["g5_csv"][1]
    assert abs(float(row[5]) - float(r["scaled_kl"])) <= 1e-6 * abs(float(row[5]))
    assert abs(float(row[6]) - float(r["ce"])) <= 1e-6
    _digest_close(param_digest(m), G["g5_param_digest"])
    np.testing.assert_allclose(m.fc2.mu_weight.detach().numpy(), A["g5_fc2_mu_weight"],
                               rtol=0, atol=1e-7)


def test_g6_eval_and_predict_match_reference():
    m = _models()["multimodal_model"]
    batches = make_batches(SEED_DATA, 2, B=2, S_opt=64, S_son=64)
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 1))
    opt = torch.optim.Adam(m.parameters(), lr=5e-5)
    crit = torch.nn.CrossEntropyLoss()
    for b in batches:  # reproduce G5's training first (the reference evaluated that model)
        loops_ref.train_step_multimodal(m, b["main_image"], b["bathy_image"], b["sss_image"],
                                        b["label"], crit, opt, 0, 2, 2, 2)
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 2))
    tot, correct, pu, mu = 0.0, 0, [], []
    for b in batches:
        r = loops_ref.eval_batch_multimodal(m, b["main_image"], b["bathy_image"], b["sss_image"],
                                            b["label"], 0, 2, 3, len(batches))
        tot += float(r["loss"])
        correct += r["correct"]
        pu += r["predictive_uncertainty"].tolist()
        mu += r["model_uncertainty"].tolist()
    row = G["g6_eval_csv"][1]
    assert abs(float(row[2]) - tot / 2) <= 1e-6 * abs(tot / 2)
    assert float(row[3]) == correct / 4
    assert abs(float(row[4]) - np.mean(pu)) <= 1e-6
    assert abs(float(row[5]) - np.mean(mu)) <= 1e-6
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 3))
    rows = []
    for i, b in enumerate(batches):
        pred, var, alea, _ = loops_ref.predict_batch(m, b["main_image"], b["bathy_image"],
                                                     b["sss_image"], 4)
        rows += [[f"img{i}_{j}", int(pred[j]), float(var[j]), float(alea[j])] for j in range(2)]
    for got, ref in zip(rows, G["g6_predict_csv"][1:]):
        assert got[0] == ref[0] and got[1] == int(ref[1])
        assert abs(got[2] - float(ref[2])) <= 1e-7 + 1e-5 * abs(float(ref[2]))
        assert abs(got[3] - float(ref[3])) <= 1e-6


def test_g7_unimodal_train_matches_reference():
    uni = _models()["image_model"]
    batches = make_batches(SEED_DATA, 2, B=2, S_opt=64, S_son=64)
    bayes_ref.set_eps_source(eps_generator_source(SEED_EPS + 4))
    opt = torch.optim.Adam(uni.parameters(), lr=1e-5)
    crit = torch.nn.CrossEntropyLoss()
    total, correct = 0.0, 0
    for b in batches:
        r = loops_ref.train_step_unimodal(uni, b["main_image"], b["label"], crit, opt, 1, 3, 2, 2)
        total += float(r["loss"])
        correct += r["correct"]
    assert abs(total / 4 - G["g7_loss"]) <= 1e-6 * abs(G["g7_loss"])
    assert correct / 4 == G["g7_acc"]
    _digest_close(param_digest(uni), G["g7_param_digest"])


def test_rho_gradient_uses_last_eps():
    """bayesian-torch aliasing: with several MC forwards before one backward, every pass's
    rho-gradient sees the LAST epsilon drawn (the behaviour mauv reproduces by default)."""
    from oracle.bayes_ref import Conv2dReparameterization
    torch.manual_seed(0)
    layer = Conv2dReparameterization(2, 3, 3, bias=False)
    layer.dnn_to_bnn_flag = True
    x = torch.randn(1, 2, 5, 5)
    eps = [torch.randn(3, 2, 3, 3) for _ in range(2)]
    it = iter(eps)
    bayes_ref.set_eps_source(lambda l, n, s: next(it))
    (layer(x).sum() + 2 * layer(x).sum()).backward()
    W = torch.zeros(3, 2, 3, 3, requires_grad=True)
    torch.nn.functional.conv2d(x, W).sum().backward()
    sig = torch.sigmoid(layer.rho_kernel.detach())
    last = 3 * W.grad * eps[1] * sig
    assert torch.allclose(layer.rho_kernel.grad, last, atol=1e-5)


def test_g10_uifm_degradation_matches_reference():
    """oracle/staging_ref.simulate_underwater_degradation == the reference's own function
    (golden_staging.npz, made by running it from the Examples script)."""
    from oracle.staging_ref import simulate_underwater_degradation as sim
    S = np.load(os.path.join(HERE, "golden_staging.npz"))
    clean, dmap = torch.from_numpy(S["clean"]), torch.from_numpy(S["dmap"])
    ones = torch.ones_like(dmap)
    for i, (turb, depth) in enumerate(((0.3, 1), (1.5, 1), (0.9, 2.5))):
        np.testing.assert_array_equal(sim(clean, ones, turb, depth).numpy(), S[f"uniform_{i}"])
        np.testing.assert_array_equal(sim(clean, dmap, turb, depth).numpy(), S[f"map_{i}"])


def test_to_tensor_normalize_known_answers():
    """ToTensor is k / 255 in fp32 for every uint8 k; Normalize is (x - mean) / std."""
    from oracle.staging_ref import to_tensor_normalize
    t = torch.arange(256, dtype=torch.uint8).view(1, 16, 16, 1)
    x = to_tensor_normalize(t)
    assert torch.equal(x.flatten(), torch.arange(256, dtype=torch.float32) / 255)
    y = to_tensor_normalize(t.expand(1, 16, 16, 3).contiguous(), (0.2, 0.3, 0.4), (0.5, 0.6, 0.7))
    assert torch.equal(y[0, 1], (x[0, 0] - torch.tensor(0.3)) / torch.tensor(0.6))
