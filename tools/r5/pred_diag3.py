"""Diagnostic of test_predictor_f16_vs_torch_autocast[224-256px] (round 5, after conv_expand16):
the HIP f16 predictor's per-item aleatoric deviation from the fp32 oracle with each 16-bit
kernel route switched off in turn (fold, expand16, big16, halo3), beside torch-autocast's, on
one fitted model."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402
from oracle import loops_ref  # noqa: E402
from tests.golden.common import make_batches, SEED_DATA  # noqa: E402
from tests.helpers import build_pair, EpsBridge, oracle_replay, fit_model  # noqa: E402


def main(S_opt=224, S_son=256, B=16, N=8):
    from mauv import engine, ops
    from mauv.engine import root_state
    from mauv.predict import mc_statistics
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
    da_a = (aa.double().cpu() - alea32.double()).abs()
    print(f"autocast: mean {da_a.mean():.3e} max {da_a.max():.3e}")
    arms = [("default", {}), ("fold off", {"FOLD": False}), ("expand16 off", {"expand16": 0}),
            ("big16 off", {"big16": 0}), ("halo3 off", {"halo3": 0}),
            ("all off", {"FOLD": False, "expand16": 0, "big16": 0, "halo3": 0})]
    for name, sw in arms:
        prev = {}
        for k, v in sw.items():
            if hasattr(engine, k):
                prev[k] = getattr(engine, k)
                setattr(engine, k, v)
            else:
                prev[k] = getattr(ops, "set_" + k)(v)
        root_state(m).eps_provider = bridge.provider
        with torch.no_grad(), torch.autocast("cuda"):
            st = mc_statistics(m, *cu, N, chunk=N)
        for k, v in prev.items():
            if hasattr(engine, k):
                setattr(engine, k, v)
            else:
                getattr(ops, "set_" + k)(v)
        da_h = (st["aleatoric"].double().cpu() - alea32.double()).abs()
        dv_h = (st["var"].double().cpu() - var32.double()).abs()
        print(f"{name:14s}: aleatoric dev mean {da_h.mean():.3e} max {da_h.max():.3e}; "
              f"var dev mean {dv_h.mean():.3e}", flush=True)
    print("aleatoric fp32 per item:", " ".join(f"{v:.3f}" for v in alea32.tolist()))


if __name__ == "__main__":
    main()
