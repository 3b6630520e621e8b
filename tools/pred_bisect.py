"""Bisect of the f16 predictor's aleatoric deviation: where in the common
f16 path does the HIP predictor's extra error against the fp32 oracle arise?

One fitted model (as test_predictor_f16_vs_torch_autocast[224-256px]), one epsilon record.
Trunk features [N, B, 2048] of each trunk are taken from three implementations:
  F32  the oracle in fp32 on the GPU (truth for this bisect),
  AC   the oracle under torch.autocast(f16) (the reference's predictor scheme),
  HIP  this library's f16 trunks (run_trunk_mc under autocast).
and fed into two heads: the oracle's head in fp32 and under autocast (f16 linears), plus the
HIP head (fp32) on HIP features (the product path).  Per combination: the per-item aleatoric /
variance deviation from the fp32 reference, and the logit error split into its per-sample
common mode and the class-relative part (the part the softmax sees).  Then per-trunk swaps
(HIP features for one trunk, F32 for the others).

Tool, not a test: prints a table (profiles/round6/pred_bisect.log)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from oracle import loops_ref  # noqa: E402
from tests.golden.common import make_batches, SEED_DATA  # noqa: E402
from tests.helpers import build_pair, EpsBridge, oracle_replay, fit_model  # noqa: E402

TRUNKS = ("image_model_feat", "bathy_model_feat", "sss_model_feat")


class Feed(torch.nn.Module):
    """Stands in for a trunk: returns the stored features of the k-th call."""

    def __init__(self, feats):
        super().__init__()
        self.feats, self.k = feats, 0

    def forward(self, x):
        f = self.feats[self.k].float()
        self.k += 1
        return f


def stats(logits):
    """[N, B, C] logits -> (aleatoric [B], variance [B]) with predictors.py:73-80's maths in
    float64 (the softmax of the given logits, whatever their dtype)."""
    P = F.softmax(logits.double(), dim=-1)
    var = torch.var(P, dim=0).mean(dim=1)
    alea = torch.mean(-torch.sum(P * torch.log(P + 1e-7), dim=-1), dim=0)
    return alea, var


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S-opt", type=int, default=224)
    ap.add_argument("--S-son", type=int, default=256)
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--N", type=int, default=8)
    ap.add_argument("--seeds", type=int, default=0,
                    help="light mode: K (data, epsilon) seeds, product vs autocast only")
    ap.add_argument("--no-fit", action="store_true", help="random-init model (no fit_model)")
    ap.add_argument("--centre", type=int, default=1, help="engine.CENTRE_Y (1 default)")
    a = ap.parse_args()
    from mauv import engine as _engine
    _engine.CENTRE_Y = bool(a.centre)
    if a.seeds:
        return sweep(a)
    from mauv import engine
    from mauv.engine import root_state, run_trunk_mc, HeadRunner
    B, N = a.B, a.N
    o, m = build_pair()
    batch = make_batches(SEED_DATA + 1, 1, B=B, S_opt=a.S_opt, S_son=a.S_son)[0]
    x, b, s = batch["main_image"], batch["bathy_image"], batch["sss_image"]
    cu = [t.cuda() for t in (x, b, s)]
    fit_model(m, *cu, torch.randint(0, 7, (B,), generator=torch.Generator().manual_seed(3)).cuda())
    o.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    bridge = EpsBridge(o, m, 7)
    with bridge:
        _, _, alea_cpu, _ = loops_ref.predict_batch(o, x, b, s, N)
    bridge.collect()

    def oracle_run(amp, feats=None):
        """logits [N,B,C] (float64, CPU) and the trunk features [N,B,2048] per trunk."""
        cap = {t: [] for t in TRUNKS}

        def fn(mm):
            hooks = []
            for t in TRUNKS:
                if feats is not None:
                    setattr(mm, t, Feed(feats[t]))
                else:
                    hooks.append(getattr(mm, t).register_forward_hook(
                        lambda mod, i, out, t=t: cap[t].append(out.detach())))
            outs = []
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16, enabled=amp):
                for _ in range(N):
                    outs.append(mm(*cu).detach())
            for h in hooks:
                h.remove()
            return torch.stack(outs)
        _, lg = oracle_replay(o, bridge.store, fn, device="cuda")
        return lg.double().cpu(), {t: torch.stack(v) for t, v in cap.items()} if feats is None \
            else None

    lg32, f32 = oracle_run(False)
    lgac, fac = oracle_run(True)
    st = root_state(m)
    st.eps_provider = bridge.provider
    fhip = {}
    with torch.no_grad(), torch.autocast("cuda"):
        for t, xx in zip(TRUNKS, cu):
            fhip[t] = run_trunk_mc(getattr(m, t), xx, N, st, 0)
        lghip = m.mc_forward(*cu, N).double().cpu()

    def hip_head(feats):
        hp = [p for n, p in m.named_parameters() if not n.split(".")[0].endswith("_feat")]
        with torch.no_grad():
            r = HeadRunner(m, st, N, 0, False)
            return engine._run(r, hp, tuple(feats[t].float().contiguous() for t in TRUNKS),
                               False).double().cpu()

    alea_ref, var_ref = stats(lg32)
    print(f"S={a.S_opt}/{a.S_son} B={B} N={N}; fp32 oracle on GPU vs CPU: aleatoric max "
          f"|d| {(alea_ref - alea_cpu.double()).abs().max():.2e}")
    print("features: relative L2 error vs F32 per trunk (per MC sample, mean over samples)")
    for t in TRUNKS:
        r = f32[t].double()
        for name, fe in (("AC", fac), ("HIP", fhip)):
            e = ((fe[t].double() - r).flatten(1).norm(dim=1) / r.flatten(1).norm(dim=1)).mean()
            bias = ((fe[t].double() - r).mean() / r.abs().mean())
            print(f"  {t:17s} {name:4s} rel L2 {e:.3e}  mean bias / mean|f| {bias:+.2e}")

    def report(tag, lg):
        al, va = stats(lg)
        da = (al - alea_ref).abs()
        dv = (va - var_ref).abs()
        d = lg - lg32
        common = d.mean(dim=-1, keepdim=True)
        rel = d - common
        print(f"  {tag:34s} alea |d| mean {da.mean():.3e} max {da.max():.3e} | var |d| mean "
              f"{dv.mean():.3e} | logit |d| mean {d.abs().mean():.3e} common {common.abs().mean():.3e}"
              f" class-rel {rel.abs().mean():.3e}")
    print("combinations (features -> head):")
    report("F32 -> fp32 head (= reference)", lg32)
    report("AC  -> autocast head (= autocast)", lgac)
    report("HIP -> HIP head (= product)", lghip)
    report("F32 -> HIP head", hip_head(f32))
    report("AC  -> HIP head", hip_head(fac))
    report("HIP -> fp32 oracle head", oracle_run(False, fhip)[0])
    report("AC  -> fp32 oracle head", oracle_run(False, fac)[0])
    report("HIP -> autocast head", oracle_run(True, fhip)[0])
    report("F32 -> autocast head", oracle_run(True, f32)[0])
    for t in TRUNKS:
        mix = dict(f32)
        mix[t] = fhip[t]
        report(f"HIP {t[:5]} only -> fp32 head", oracle_run(False, mix)[0])
        mix[t] = fac[t]
        report(f"AC  {t[:5]} only -> fp32 head", oracle_run(False, mix)[0])
    print("aleatoric fp32 per item:", " ".join(f"{v:.3f}" for v in alea_ref.tolist()))


def sweep(a):
    """Per (data, epsilon) seed: the per-item aleatoric and predictive-entropy deviations of the
    HIP f16 predictor and of torch-autocast from the fp32 oracle (GPU), on one fitted model per
    data seed."""
    from mauv.engine import root_state
    from mauv.predict import mc_statistics
    B, N = a.B, a.N
    rows = []
    for k in range(a.seeds):
        o, m = build_pair()
        batch = make_batches(SEED_DATA + 1 + k, 1, B=B, S_opt=a.S_opt, S_son=a.S_son)[0]
        x, b, s = batch["main_image"], batch["bathy_image"], batch["sss_image"]
        cu = [t.cuda() for t in (x, b, s)]
        if not a.no_fit:
            fit_model(m, *cu, torch.randint(0, 7, (B,),
                                            generator=torch.Generator().manual_seed(3 + k)).cuda())
            o.load_state_dict({kk: v.cpu() for kk, v in m.state_dict().items()})
        bridge = EpsBridge(o, m, 7 + 100 * k)
        with bridge, torch.no_grad():
            for _ in range(N):
                o(*[t[:1] for t in (x, b, s)])
        bridge.collect()

        def run(mm, amp):
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16, enabled=amp):
                return torch.stack([mm(*cu) for _ in range(N)]).double().cpu()
        _, lg32 = oracle_replay(o, bridge.store, lambda mm: run(mm, False), device="cuda")
        _, lgac = oracle_replay(o, bridge.store, lambda mm: run(mm, True), device="cuda")
        root_state(m).eps_provider = bridge.provider
        with torch.no_grad(), torch.autocast("cuda"):
            st = mc_statistics(m, *cu, N, chunk=N)

        def pent(lg):
            pm = F.softmax(lg, -1).mean(0)
            return -(pm * torch.log(pm + 1e-8)).sum(-1)
        ar, vr = stats(lg32)
        aa, va_ = stats(lgac)
        dvh = (st["var"].double().cpu() - vr).abs()
        dva = (va_ - vr).abs()
        print(f"seed {k}: variance |d| mean HIP {dvh.mean():.3e} autocast {dva.mean():.3e}, max "
              f"HIP {dvh.max():.3e} autocast {dva.max():.3e} (|var| <= {vr.abs().max():.3e})")
        dah = (st["aleatoric"].double().cpu() - ar).abs()
        daa = (aa - ar).abs()
        dph = (st["predictive_entropy"].double().cpu() - pent(lg32)).abs()
        dpa = (pent(lgac) - pent(lg32)).abs()
        root_state(m).eps_provider = bridge.provider
        with torch.no_grad(), torch.autocast("cuda"):
            lh = m.mc_forward(*cu, N).double().cpu()
        bar = 5e-2 * lg32.abs().clamp(min=1)
        vh = int(((lh - lg32).abs() > bar).sum())
        va = int(((lgac - lg32).abs() > bar).sum())
        rows.append((dah.mean().item(), daa.mean().item(), dah.max().item(), daa.max().item(),
                     dph.max().item(), dpa.max().item(), vh, va, (lh - lg32).abs().max().item(),
                     (lgac - lg32).abs().max().item(), dph.mean().item(), dpa.mean().item()))
        print(f"seed {k}: aleatoric |d| mean HIP {rows[-1][0]:.3e} autocast {rows[-1][1]:.3e} "
              f"(ratio {rows[-1][0] / rows[-1][1]:.2f}); max HIP {rows[-1][2]:.3e} autocast "
              f"{rows[-1][3]:.3e}; predictive entropy max HIP {rows[-1][4]:.3e} autocast "
              f"{rows[-1][5]:.3e} (mean {rows[-1][10]:.3e} / {rows[-1][11]:.3e}); logits over "
              f"SURVEY's 5e-2 max(1,|ref|) HIP {vh} autocast {va} of {lg32.numel()} (max |d| "
              f"{rows[-1][8]:.3e} / {rows[-1][9]:.3e}, |ref| <= {lg32.abs().max():.1f}); classes "
              f"{len(set(F.softmax(lg32, -1).mean(0).argmax(-1).tolist()))}", flush=True)
        del o, m
        torch.cuda.empty_cache()
    import numpy as np
    r = np.array(rows)
    print(f"over {len(rows)} seeds: mean-of-means HIP {r[:, 0].mean():.3e} autocast "
          f"{r[:, 1].mean():.3e} (ratio {r[:, 0].mean() / r[:, 1].mean():.2f}); ratio per seed "
          f"min {np.min(r[:, 0] / r[:, 1]):.2f} max {np.max(r[:, 0] / r[:, 1]):.2f}; worst item "
          f"HIP {r[:, 2].max():.3e} autocast {r[:, 3].max():.3e}; predictive entropy mean "
          f"HIP {r[:, 10].mean():.3e} autocast {r[:, 11].mean():.3e}, worst HIP {r[:, 4].max():.3e} "
          f"autocast {r[:, 5].max():.3e}; logit bar violations HIP {int(r[:, 6].sum())} autocast "
          f"{int(r[:, 7].sum())}")


if __name__ == "__main__":
    main()
