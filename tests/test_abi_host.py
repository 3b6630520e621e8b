"""CPU checks: the C-ABI library loads and exports every symbol include/mauv.h declares; host
logic (state_dict compatibility, MOPED init, known answers, checkpoint key rewrites, Philox
known-answer vectors, KL table packing).  No compute calls — there is no GPU here."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "mauv.h")


def header_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_ ]+\**\s+\**(mauv_\w+)\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    from mauv._lib import LIB_PATH, SIGNATURES
    lib = ctypes.CDLL(LIB_PATH)
    names = header_functions()
    assert len(names) >= 30, names
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/mauv.h but not exported"
    assert set(SIGNATURES) == set(names), set(SIGNATURES) ^ set(names)


def test_ctypes_arity_matches_header():
    """Every prototype's parameter count in include/mauv.h equals the ctypes argtypes."""
    from mauv._lib import SIGNATURES
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    protos = dict(re.findall(r"(mauv_\w+)\(([^)]*)\)\s*;", txt))
    for name, params in protos.items():
        params = params.strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        assert len(SIGNATURES[name]) == n, (name, n, len(SIGNATURES[name]))


def test_library_reports_gfx950_only():
    from mauv._lib import LIB_PATH
    out = os.popen(f"/opt/rocm/lib/llvm/bin/llvm-readelf -n {LIB_PATH} 2>/dev/null | head -0; "
                   f"strings -a {LIB_PATH} | grep -o 'amdgcn-amd-amdhsa--gfx[0-9a-z]*' | sort -u"
                   ).read().split()
    assert out and all(t.endswith("gfx950") for t in out), out


def test_abi_version_and_error_string():
    from mauv._lib import lib
    assert lib.mauv_abi_version() == 4
    assert isinstance(lib.mauv_last_error(), bytes)


def test_route_host_record():
    """MauvRoute (include/mauv.h) is host-only state: the measured defaults, get / set round
    trips through the ctypes Structure, and an invalid field changes nothing."""
    from mauv import ops
    from mauv._lib import lib, MauvRoute
    assert ctypes.sizeof(MauvRoute) == 16 * 4
    r = ops.route()
    if "MAUV_F32_MATH" not in os.environ:
        assert r["f32_math"] == 6
    assert (r["halo3"], r["big16"], r["big16_min_k"], r["haloc16"], r["expand16"],
            r["reparam_kernels"]) == (1, 1, 512, 1, 1, 3)
    ops.set_f32_math("exact")
    try:
        assert ops.f32_math() == "exact"
        assert ops.set_f32_math("split3") == "exact"
        with pytest.raises(RuntimeError, match="f32_math"):
            ops.set_route(f32_math=7)
        with pytest.raises(RuntimeError, match="haloc16"):
            ops.set_route(halo3=0, haloc16=9)   # rejected as a whole: halo3 stays 1
        assert ops.route()["halo3"] == 1 and ops.f32_math() == "split3"
        assert ops.set_expand16(3) == 1 and ops.set_expand16(None) == 3
        assert ops.set_big16(True, 1024) == 1 and ops.route()["big16_min_k"] == 1024
        with pytest.raises(RuntimeError, match="big16_min_k"):
            ops.set_big16(True, 256)    # below the K range conv_big16 is tested on
        with pytest.raises(ValueError):
            ops.set_route(dma16=1)
        bad = MauvRoute()
        assert lib.mauv_get_route(ctypes.byref(bad)) == 0
        bad.reparam_kernels = 4
        assert lib.mauv_set_route(ctypes.byref(bad)) < 0 and b"reparam" in lib.mauv_last_error()
    finally:
        ops.set_route(**r)
    assert ops.route() == r


def test_state_dict_compatible_with_reference_layout():
    from mauv.models import define_models, DEFAULT_PRIOR
    from oracle.model_ref import define_models as oracle_define
    torch.manual_seed(0)
    m = define_models(None, 7, DEFAULT_PRIOR)
    torch.manual_seed(0)
    o = oracle_define(None, 7, DEFAULT_PRIOR)
    for k in m:
        a, b = m[k].state_dict(), o[k].state_dict()
        assert list(a) == list(b), k
        for n in a:
            assert a[n].shape == b[n].shape and torch.equal(a[n], b[n]), (k, n)
    mm = m["multimodal_model"]
    assert sum(p.numel() for p in mm.parameters()) == 146_767_638
    assert sum(p.numel() for n, p in mm.named_parameters() if "mu_" in n) == 73_304_139
    assert sum(p.numel() for n, p in m["image_model"].named_parameters() if "mu_" in n) \
        == 23_469_255


def test_moped_rho_and_prior():
    from mauv.layers import dnn_to_bnn, Conv2dReparameterization, LinearReparameterization
    net = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3, bias=False), torch.nn.Linear(4, 2))
    w = net[0].weight.detach().clone()
    dnn_to_bnn(net, {"prior_mu": 0.0, "prior_sigma": 1.0, "posterior_mu_init": 0.0,
                     "posterior_rho_init": -3.0, "moped_enable": True, "moped_delta": 0.1})
    assert isinstance(net[0], Conv2dReparameterization) and isinstance(net[1], LinearReparameterization)
    assert torch.equal(net[0].mu_kernel.detach(), w)
    assert torch.allclose(net[0].rho_kernel.detach(), torch.log(torch.expm1(0.1 * w.abs()) + 1e-20))
    assert net[0].dnn_to_bnn_flag and net[1].prior_variance == 1.0
    dnn_to_bnn(net, {"prior_mu": 0.0, "prior_sigma": 1.0, "posterior_mu_init": 0.0,
                     "posterior_rho_init": -3.0, "moped_enable": True, "moped_delta": 0.1})
    assert isinstance(net[0], Conv2dReparameterization)  # idempotent


def test_checkpoint_key_rewrites():
    from mauv.checkpointing import remap_keys
    keys = {"image_model_feat.conv1.mu_kernel": (64, 3, 7, 7), "fc2.mu_weight": (7, 32)}
    sd = {"module.image_model_feat.model.conv1.mu_kernel": torch.zeros(64, 3, 7, 7),
          "fc2.mu_weight": torch.zeros(5, 32), "junk": torch.zeros(1)}
    out, skipped = remap_keys(sd, keys)
    assert list(out) == ["image_model_feat.conv1.mu_kernel"]
    assert len(skipped) == 2 and any("shape mismatch" in s for s in skipped)


def test_philox_known_answers():
    """Random123 Philox4x32-10 known-answer vectors (the generator behind every epsilon)."""
    from oracle.philox_ref import philox4x32_10
    r = philox4x32_10(np.array([0], dtype=np.uint64), 0, 0, 0)[0]
    assert [hex(v) for v in r] == ["0x6627e8d5", "0xe169c58d", "0xbc57ac4c", "0x9b00dbd8"]
    # counter (0xffffffff x4), key (0xffffffff x2)
    r = philox4x32_10(np.array([0xFFFFFFFF], dtype=np.uint64), 0xFFFFFFFFFFFFFFFF, 0xFFFFFFFF,
                      0xFFFFFFFFFFFFFFFF)[0]
    assert [hex(v) for v in r] == ["0x408f276d", "0x41c83b0e", "0xa20bc7c6", "0x6d5451fd"]


def test_kl_table_packing():
    from mauv.kl import KLTable
    from mauv.layers import LinearReparameterization
    lin = LinearReparameterization(4, 3, prior_mean=0.25, prior_variance=2.0)
    tab = KLTable([lin])
    rows = tab._build(False, "cpu").numpy()
    assert rows.shape == (2, 6) and rows[0, 4] == 12 and rows[1, 4] == 3
    pm, ps = rows[0, 5:6].view(np.float32)
    assert (pm, ps) == (0.25, 2.0)
    assert rows[0, 0] == lin.mu_weight.data_ptr() and rows[1, 1] == lin.rho_bias.data_ptr()


def test_engine_layer_ids_and_sample_counter():
    from mauv.models import define_models, DEFAULT_PRIOR
    from mauv.engine import root_state
    m = define_models(None, 7, DEFAULT_PRIOR)["multimodal_model"]
    st = root_state(m)
    assert len(st.ids) == 174  # 159 convs + 15 linears
    assert len(set(st.ids.values())) == 174
    assert st.next_samples(5) == 0 and st.next_samples(1) == 5 and st.offset == 6


def test_mc_shard_counts():
    from mauv.predict import local_mc_count
    for n in (1, 5, 100, 101):
        for w in (1, 2, 3, 8):
            counts = [local_mc_count(n, r, w) for r in range(w)]
            assert sum(counts) == n and max(counts) - min(counts) <= 1


def _trunk_convs(S, B=64):
    """(H, Cin, Cout, R, stride) of every ResNet-50 conv after the stem, at input size S."""
    H, inp, out = S // 4, 64, []
    for planes, blocks, st in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for bi in range(blocks):
            s = st if bi == 0 else 1
            out += [(H, inp, planes, 1, 1), (H, planes, planes, 3, s), (H // s, planes, planes * 4, 1, 1)]
            if bi == 0:
                out.append((H, inp, planes * 4, 1, s))
            H, inp = H // s, planes * 4
    return out


def _wgrad_cost_argmin(G, B, H, Cin, Cout, R, st):
    """Restatement of mauv_conv2d_wgrad_splits' default rule (MAUV_WGRAD_SPLITS=2): block rounds
    x the per-block MFMA time of a pixel chunk + the fp32 slab bytes written and read back."""
    pad = R // 2
    Ho = (H + 2 * pad - R) // st + 1
    P = B * Ho * Ho
    N = R * R * Cin
    tm, tn = (64 if Cout <= 64 else 128), (64 if N <= 64 else 128)
    tiles = -(-Cout // tm) * -(-N // tn) * G
    maxs = max(1, min(256, (P + 255) // 256))
    best, tbest = 1, 1e30
    for s in range(1, maxs + 1):
        nb = tiles * s
        rounds = -(-nb // 512)
        kch = (-(-P // s) + 31) // 32 * 32
        t = rounds * (kch * 2.0 * tm * tn / (480e12 / 512) + 2e-6) + nb * tm * tn * 8.0 / 5e12
        if t < tbest * 0.995:
            best, tbest = s, t
    return best, tiles


def test_wgrad_split_count_prices_slab_bytes():
    """mauv_conv2d_wgrad_splits (host helper, conv_gemm.hip): the default split count is the
    argmin of block rounds x chunk time + slab bytes (restated above) for every weight gradient
    of the three trunks at the bench workload, and it writes at most 60 % of the fp32 slab bytes
    of the round-filling rule (MAUV_WGRAD_SPLITS=1: one to three rounds, last round >= 80 % full);
    the round-1 rule (=0, the fewest splits giving >= 1024 blocks) still answers in a fresh
    process."""
    import subprocess
    import sys
    from mauv import ops
    convs = [(H, Cin, Cout, R, st) for S in (224, 256) for H, Cin, Cout, R, st in _trunk_convs(S)]
    slab2 = 0
    for H, Cin, Cout, R, st in convs:
        sp = ops.wgrad_splits(5, 64, H, H, Cin, Cout, R, st, R // 2)
        want, tiles = _wgrad_cost_argmin(5, 64, H, Cin, Cout, R, st)
        assert sp == want, (H, Cin, Cout, R, st, sp, want)
        slab2 += sp * tiles
    code = ("import sys; sys.path[:0] = [%r, %r]; from mauv import ops; "
            "print(' '.join(str(ops.wgrad_splits(5, 64, H, H, Ci, Co, R, st, R // 2)) "
            "for H, Ci, Co, R, st in %r))"
            % (REPO, os.path.join(REPO, "multimodal-auv_amd"), convs))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True,
                         env=dict(os.environ, MAUV_WGRAD_SPLITS="1")).stdout.split()
    slab1 = 0
    for (H, Cin, Cout, R, st), sp in zip(convs, map(int, out[-len(convs):])):
        tiles = _wgrad_cost_argmin(5, 64, H, Cin, Cout, R, st)[1]
        nb = tiles * sp
        rounds = -(-nb // 512)
        assert 1 <= rounds <= 3 and nb / (rounds * 512) >= 0.8, (H, Cin, Cout, R, st, sp, nb)
        slab1 += nb
    assert slab2 <= 0.6 * slab1, (slab2, slab1)
    code = ("import sys; sys.path[:0] = [%r, %r]; from mauv import ops; "
            "print(ops.wgrad_splits(5, 64, 64, 64, 64, 64, 3, 1, 1))"
            % (REPO, os.path.join(REPO, "multimodal-auv_amd")))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True,
                         env=dict(os.environ, MAUV_WGRAD_SPLITS="0")).stdout.split()[-1]
    assert int(out) == 41   # ceil(1024 / 25 tiles)


def test_m16_magic_division_exact():
    """conv_common.h m16_div / udiv16 (the weight-gradient loaders' pixel -> (row, image)
    carry): q = umulhi(n, floor((2^32 - 1) / d) + 1) equals n // d for every n < 2^17 and
    2 <= d <= 4096 (d = 1 takes the m = 0 path, q = n)."""
    n = np.arange(1 << 17, dtype=np.uint64)
    for d in range(2, 4097):
        m = np.uint64((0xFFFFFFFF // d) + 1)
        assert np.array_equal((n * m) >> np.uint64(32), n // np.uint64(d)), d
