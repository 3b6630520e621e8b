"""Which f16 rounding points carry the f16 predictor's error (second step)?

The oracle model runs in fp32 on the GPU (TF32 off) with f16 rounding (RNE, torch's .half())
emulated at chosen points of every Bayesian conv / BN / bottleneck:
  in   the conv input (the stored activation the next conv reads; images for the stems)
  w    the sampled weight
  y    the conv output before its BatchNorm (what both f16 schemes store)
  bn   the BatchNorm output (torch-autocast rounds it; this library folds BN into the consumer
       and rounds once there, which 'in' already models)
  blk  the bottleneck output relu(bn3 + identity)
  feat the pooled trunk features (autocast: f16; this library: fp32)
  yc   the conv output stored as f16(y - c) + c, c = its BatchNorm's running mean at the call
       (replaces 'y': the storage error then scales with |y - c| ~ the batch spread instead of
       |y|, which BatchNorm's 1/std amplifies when the channel mean is large)
All points on = torch-autocast's scheme; every point but bn / feat = this library's.  Each
configuration is compared with the exact fp32 run (same weights, same epsilons) on a fitted
model: per-trunk feature relative L2 error and the per-item aleatoric deviation.  The library's
own f16 path is printed beside them.  Tool, not a test (profiles/round6/f16_rounding_points.log).
"""
import contextlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "multimodal-auv_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from oracle import resnet_ref  # noqa: E402
from tests.golden.common import make_batches, SEED_DATA  # noqa: E402
from tests.helpers import build_pair, EpsBridge, oracle_replay, fit_model  # noqa: E402

TRUNKS = ("image_model_feat", "bathy_model_feat", "sss_model_feat")
POINTS = ("in", "w", "y", "bn", "blk", "feat")   # + "yc" (not part of either scheme)


def r16(t):
    return t.half().float()


@contextlib.contextmanager
def rounding(points, trunk_mods):
    """Patch F.conv2d / F.batch_norm and hook the bottlenecks / trunks for the given points
    (trunk convs only: the head is fp32 in both comparisons here)."""
    conv0, bn0 = F.conv2d, F.batch_norm
    active = {"on": False}

    def conv(x, w, *a, **k):
        if not active["on"] or x.dim() != 4:
            return conv0(x, w, *a, **k)
        if "in" in points:
            x = r16(x)
        if "w" in points:
            w = r16(w)
        y = conv0(x, w, *a, **k)
        return r16(y) if "y" in points else y

    def bn(x, *a, **k):
        if active["on"] and "yc" in points and a and a[0] is not None:
            c = a[0].detach().view(1, -1, 1, 1)
            x = r16(x - c) + c
        out = bn0(x, *a, **k)
        return r16(out) if active["on"] and "bn" in points else out
    hooks = []
    for tm in trunk_mods:
        hooks.append(tm.register_forward_pre_hook(lambda m, i: active.__setitem__("on", True)))
        hooks.append(tm.register_forward_hook(
            lambda m, i, o: (active.__setitem__("on", False),
                             r16(o) if "feat" in points else o)[1]))
        for mod in tm.modules():
            if isinstance(mod, resnet_ref.Bottleneck) and "blk" in points:
                hooks.append(mod.register_forward_hook(lambda m, i, o: r16(o)))
    F.conv2d, F.batch_norm = conv, bn
    try:
        yield
    finally:
        F.conv2d, F.batch_norm = conv0, bn0
        for h in hooks:
            h.remove()


def stats(lg):
    P = F.softmax(lg.double(), -1)
    return torch.mean(-torch.sum(P * torch.log(P + 1e-7), dim=-1), dim=0)


def main(S_opt=224, S_son=256, B=16, N=8, seeds=(0, 1, 2)):
    from mauv.engine import root_state, run_trunk_mc
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    configs = [("exact fp32", ()),
               ("autocast-like (all)", POINTS),
               ("library-like (in w y blk)", ("in", "w", "y", "blk")),
               ("only in", ("in",)), ("only w", ("w",)), ("only y", ("y",)),
               ("only blk", ("blk",)), ("in w y blk, not in", ("w", "y", "blk")),
               ("in w y blk, not w", ("in", "y", "blk")),
               ("in w y blk, not y", ("in", "w", "blk")),
               ("in w yc blk (centred y)", ("in", "w", "yc", "blk"))]
    acc = {name: [[], {t: [] for t in TRUNKS}] for name, _ in configs + [("library (HIP)", ())]}
    for k in seeds:
        o, m = build_pair()
        batch = make_batches(SEED_DATA + 1 + k, 1, B=B, S_opt=S_opt, S_son=S_son)[0]
        x, b, s = batch["main_image"], batch["bathy_image"], batch["sss_image"]
        cu = [t.cuda() for t in (x, b, s)]
        fit_model(m, *cu, torch.randint(0, 7, (B,),
                                        generator=torch.Generator().manual_seed(3 + k)).cuda())
        o.load_state_dict({kk: v.cpu() for kk, v in m.state_dict().items()})
        bridge = EpsBridge(o, m, 7 + 100 * k)
        with bridge, torch.no_grad():
            for _ in range(N):
                o(*[t[:1] for t in (x, b, s)])
        bridge.collect()
        res = {}
        for name, pts in configs:
            cap = {t: [] for t in TRUNKS}

            def fn(mm, pts=pts, cap=cap):
                trunks = [getattr(mm, t) for t in TRUNKS]
                with torch.no_grad(), rounding(set(pts), trunks):
                    hs = [getattr(mm, t).register_forward_hook(   # after the rounding hooks
                        lambda mod, i, out, t=t: cap[t].append(out.detach().float()))
                        for t in TRUNKS]
                    lg = torch.stack([mm(*cu) for _ in range(N)])
                for h in hs:
                    h.remove()
                return lg.double().cpu()
            _, lg = oracle_replay(o, bridge.store, fn, device="cuda")
            res[name] = (lg, {t: torch.stack(v) for t, v in cap.items()})
        st = root_state(m)
        st.eps_provider = bridge.provider
        with torch.no_grad(), torch.autocast("cuda"):
            fh = {t: run_trunk_mc(getattr(m, t), xx, N, st, 0) for t, xx in zip(TRUNKS, cu)}
            lh = m.mc_forward(*cu, N).double().cpu()
        res["library (HIP)"] = (lh, fh)
        lg0, f0 = res["exact fp32"]
        a0 = stats(lg0)
        for name, (lg, fe) in res.items():
            acc[name][0].append((stats(lg) - a0).abs())
            for t in TRUNKS:
                r = f0[t].double()
                acc[name][1][t].append(((fe[t].double() - r).flatten(1).norm(dim=1) /
                                        r.flatten(1).norm(dim=1)).mean().item())
        del o, m
        torch.cuda.empty_cache()
        print(f"seed {k} done", flush=True)
    print(f"S={S_opt}/{S_son} B={B} N={N}, seeds {list(seeds)}: feature rel L2 error vs exact "
          f"fp32 (image / bathy / sss, mean over seeds) and |d aleatoric| over all items")
    for name in acc:
        da = torch.cat(acc[name][0])
        fe = " / ".join(f"{sum(v) / len(v):.3e}" for v in acc[name][1].values())
        print(f"  {name:28s} feat {fe}   alea |d| mean {da.mean():.3e} max {da.max():.3e}")


if __name__ == "__main__":
    main()
