"""Diagnostic of test_predictor_f16_vs_torch_autocast[224-256px]: per-item aleatoric / variance
deviations of the HIP f16 predictor, torch-autocast and the HIP fp32 predictor against the fp32
oracle, on models fitted with engine.BWD_PARTIALS_F32 off and on (the fitted weights differ in
the last bits of the fp32 gradient sums, which 20 Adam steps amplify)."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402
from oracle import loops_ref  # noqa: E402
from tests.golden.common import make_batches, SEED_DATA  # noqa: E402
from tests.helpers import build_pair, EpsBridge, oracle_replay, fit_model  # noqa: E402


def run(bp, S_opt=224, S_son=256, B=16, N=8):
    from mauv import engine
    from mauv.engine import root_state
    from mauv.predict import mc_statistics
    engine.BWD_PARTIALS_F32 = bp
    o, m = build_pair()
    batch = make_batches(SEED_DATA + 1, 1, B=B, S_opt=S_opt, S_son=S_son)[0]
    x, b, s = batch["main_image"], batch["bathy_image"], batch["sss_image"]
    cu = [t.cuda() for t in (x, b, s)]
    fit_model(m, *cu, torch.randint(0, 7, (B,), generator=torch.Generator().manual_seed(3)).cuda())
    o.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    bridge = EpsBridge(o, m, 7)
    with bridge:
        pred32, var32, alea32, _ = loops_ref.predict_batch(o, x, b, s, N)
    bridge.collect()

    def ac(mm):
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            return loops_ref.predict_batch(mm, *cu, N)
    _, (pa, va, aa, _) = oracle_replay(o, bridge.store, ac, device="cuda")
    root_state(m).eps_provider = bridge.provider
    with torch.no_grad(), torch.autocast("cuda"):
        st = mc_statistics(m, *cu, N, chunk=N)
    root_state(m).eps_provider = bridge.provider
    with torch.no_grad():
        st32 = mc_statistics(m, *cu, N, chunk=N)
    da_h = (st["aleatoric"].double().cpu() - alea32.double()).abs()
    da_a = (aa.double().cpu() - alea32.double()).abs()
    da_32 = (st32["aleatoric"].double().cpu() - alea32.double()).abs()
    print(f"BWD_PARTIALS_F32={bp}: aleatoric max dev HIP f16 {da_h.max():.3e} autocast {da_a.max():.3e} "
          f"HIP fp32 {da_32.max():.3e}; mean {da_h.mean():.3e} / {da_a.mean():.3e} / {da_32.mean():.3e}")
    print("  per item HIP f16:", " ".join(f"{v:.1e}" for v in da_h.tolist()))
    print("  per item autocast:", " ".join(f"{v:.1e}" for v in da_a.tolist()))
    print("  aleatoric fp32:", " ".join(f"{v:.3f}" for v in alea32.tolist()))


if __name__ == "__main__":
    run(False)
    run(True)
