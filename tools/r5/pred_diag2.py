"""Logit-level diagnostic for the f16 predictor on a fitted model: max |logit - fp32| of the HIP
f16 path (fold on / off), torch-autocast and the HIP fp32 path, per MC sample, same epsilons."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402
from tests.golden.common import make_batches, SEED_DATA  # noqa: E402
from tests.helpers import build_pair, EpsBridge, oracle_replay, fit_model  # noqa: E402


def main(S_opt=224, S_son=256, B=16, N=8):
    from mauv import engine
    from mauv.engine import root_state
    o, m = build_pair()
    batch = make_batches(SEED_DATA + 1, 1, B=B, S_opt=S_opt, S_son=S_son)[0]
    x, b, s = batch["main_image"], batch["bathy_image"], batch["sss_image"]
    cu = [t.cuda() for t in (x, b, s)]
    fit_model(m, *cu, torch.randint(0, 7, (B,), generator=torch.Generator().manual_seed(3)).cuda())
    o.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    bridge = EpsBridge(o, m, 7)
    with bridge, torch.no_grad():
        ref = torch.stack([o(x, b, s) for _ in range(N)]).double()
    bridge.collect()

    def ac(mm):
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            return torch.stack([mm(*cu) for _ in range(N)]).float()
    _, lac = oracle_replay(o, bridge.store, ac, device="cuda")
    out = {"autocast": lac.double().cpu()}
    for name, amp, fold in (("hip_f16", True, True), ("hip_f16_nofold", True, False),
                            ("hip_fp32", False, True)):
        engine.FOLD = fold
        root_state(m).eps_provider = bridge.provider
        with torch.no_grad(), torch.autocast("cuda", enabled=amp):
            out[name] = m.mc_forward(*cu, N).double().cpu()
    engine.FOLD = True
    print(f"|logit| max {ref.abs().max():.3f}, logit spread over MC {ref.std(0).mean():.4f}")
    for k, v in out.items():
        d = (v - ref).abs()
        print(f"{k:16s} max |dlogit| {d.max():.3e}  mean {d.mean():.3e}  per sample max "
              + " ".join(f"{t:.1e}" for t in d.amax((1, 2)).tolist()))


if __name__ == "__main__":
    main()
