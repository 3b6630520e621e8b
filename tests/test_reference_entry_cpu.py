"""The reference's own entry points import unchanged on the drop-in (missing 1).

`main.py`, every `Examples/*.py`, `functions/functions.py` and `cli.py` import 19 distinct
`Multimodal_AUV.*` modules.  With `MAUV_REFERENCE_PKG` pointing at the reference's
`src/Multimodal_AUV`, the on-path ones must come from the drop-in (mauv-backed) and the
off-path ones (`inference.inference_data`, `data.*`, `config.*`, `Examples.*`,
`data_preparation.*`, `functions.*`) from the reference — including modules of a drop-in
SUBpackage such as `Multimodal_AUV.inference.inference_data` (`main.py:14`,
`Examples/Example_training_from_scratch.py:17`).  The reference's documented top-level API
(`__init__.py:5-10`, used at `README - pypi.md:324,402,515,594`) must re-export.

Third-party modules the reference imports that are absent from this image (torchvision,
tensorboard, pynvml, skimage, cv2, rasterio, pyproj, utm, exiftool) get name-only shims, the
way `tests/golden/make_golden.py:48-78` installs them; nothing of theirs runs at import time.
Runs in a subprocess so the shims and the reference path never leak into other tests.  Needs
`/root/reference` (this container only; the GPU box has no reference).
"""
import ast
import json
import os
import subprocess
import sys
import textwrap

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "multimodal-auv_amd")
REF_PKG = "/root/reference/src/Multimodal_AUV"

pytestmark = pytest.mark.skipif(not os.path.isdir(REF_PKG),
                                reason="reference checkout not present")

ENTRY_FILES = ["main.py", "cli.py", "functions/functions.py"]


def _entry_files():
    ex = os.path.join(REF_PKG, "Examples")
    return ENTRY_FILES + sorted("Examples/" + f for f in os.listdir(ex)
                                if f.endswith(".py") and f != "__init__.py")


def _all_files():
    for d, _, fs in os.walk(REF_PKG):
        for f in fs:
            if f.endswith(".py"):
                yield os.path.relpath(os.path.join(d, f), REF_PKG)


def _imported_modules():
    """Every `Multimodal_AUV.*` module any reference file imports (parsed, not executed)."""
    mods = set()
    for rel in _all_files():
        tree = ast.parse(open(os.path.join(REF_PKG, rel), encoding="utf-8-sig").read())
        for node in ast.walk(tree):
            if isinstance(node, ast.ImportFrom) and node.module and \
                    node.module.startswith("Multimodal_AUV."):
                mods.add(node.module)
            elif isinstance(node, ast.Import):
                mods.update(a.name for a in node.names if a.name.startswith("Multimodal_AUV."))
    return sorted(mods)


_SCRIPT = textwrap.dedent(r'''
    import importlib, importlib.abc, importlib.machinery, importlib.util, json, os, sys, types
    sys.path[:0] = [PKG_ROOT, REPO]
    os.environ["MAUV_REFERENCE_PKG"] = REF_PKG
    os.environ.setdefault("MPLBACKEND", "Agg")

    ABSENT = ["torchvision", "tensorboard", "pynvml", "skimage", "cv2", "rasterio", "pyproj",
              "utm", "exiftool"]
    ROOTS = {r for r in ABSENT if importlib.util.find_spec(r) is None}

    class _Dummy:
        def __init__(self, *a, **k): pass
        def __call__(self, *a, **k): return _Dummy()
        def __getattr__(self, k): return _Dummy()

    class _NameOnly(types.ModuleType):
        def __getattr__(self, k):
            if k.startswith("__"):
                raise AttributeError(k)
            return _Dummy

    class _Finder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
        def find_spec(self, name, path=None, target=None):
            if name.split(".")[0] in ROOTS or name == "torch.utils.tensorboard":
                return importlib.machinery.ModuleSpec(name, self, is_package=True)
            return None
        def create_module(self, spec):
            m = _NameOnly(spec.name); m.__path__ = []; return m
        def exec_module(self, m): pass

    sys.meta_path.insert(0, _Finder())

    out = {"modules": {}, "api": {}, "entry": {}}
    for name in MODULES:
        m = importlib.import_module(name)
        out["modules"][name] = os.path.realpath(m.__file__)
    import Multimodal_AUV
    for api in ("run_auv_inference", "run_auv_retraining", "run_auv_preprocessing",
                "run_AUV_training_from_scratch"):
        ns = {}
        exec(f"from Multimodal_AUV import {api}", ns)
        out["api"][api] = ns[api].__module__
    # the entry scripts' import blocks (their bodies sit behind `if __name__ == "__main__"`)
    for rel, modname in ENTRIES:
        spec = importlib.util.spec_from_file_location(modname, os.path.join(REF_PKG, rel))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[modname] = mod
        spec.loader.exec_module(mod)
        out["entry"][rel] = {k: getattr(getattr(mod, k), "__module__", "")
                             for k in ("define_models", "multimodal_predict_and_save",
                                       "prepare_inference_datasets_and_loaders",
                                       "train_and_evaluate_multimodal_model",
                                       "move_models_to_device") if hasattr(mod, k)}
    print("RESULT " + json.dumps(out))
''')


def _run(modules, entries):
    code = (f"PKG_ROOT={PKG_ROOT!r}\nREPO={REPO!r}\nREF_PKG={REF_PKG!r}\n"
            f"MODULES={modules!r}\nENTRIES={entries!r}\n" + _SCRIPT)
    env = dict(os.environ)
    env.pop("MAUV_REFERENCE_PKG", None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       env=env, timeout=600, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def test_reference_entry_points_import_on_dropin():
    mods = _imported_modules()
    assert "Multimodal_AUV.inference.inference_data" in mods
    assert len(mods) >= 19, mods
    entries = [("main.py", "Multimodal_AUV.main"),
               ("Examples/Example_training_from_scratch.py",
                "Multimodal_AUV.Examples.Example_training_from_scratch")]
    res = _run(mods, entries)
    dropin = os.path.realpath(os.path.join(PKG_ROOT, "Multimodal_AUV"))
    ref = os.path.realpath(REF_PKG)
    on_path = {"Multimodal_AUV.models.model_utils", "Multimodal_AUV.utils.device",
               "Multimodal_AUV.train.loop_utils", "Multimodal_AUV.train.checkpointing",
               "Multimodal_AUV.inference.predictors"}
    for name, f in res["modules"].items():
        if name in on_path:
            assert f.startswith(dropin), (name, f)
        elif name.split(".")[1] in ("data", "config", "Examples", "data_preparation",
                                    "functions") or name.endswith("inference_data"):
            assert f.startswith(ref), (name, f)
    assert res["modules"]["Multimodal_AUV.inference.inference_data"].startswith(ref)
    # top-level API from the reference's functions.functions
    assert set(res["api"].values()) == {"Multimodal_AUV.functions.functions"}
    # the entry scripts bind the mauv implementations for the hot path
    for rel, names in res["entry"].items():
        assert names["define_models"] == "mauv.models", (rel, names)
        assert names["multimodal_predict_and_save"] == "mauv.predict", (rel, names)
        assert names["move_models_to_device"] == "mauv.device", (rel, names)
        assert names["prepare_inference_datasets_and_loaders"] == \
            "Multimodal_AUV.inference.inference_data", (rel, names)


def test_run_api_without_reference_is_actionable():
    code = (f"import sys; sys.path[:0]=[{PKG_ROOT!r}, {REPO!r}]\n"
            "import Multimodal_AUV\n"
            "try:\n    from Multimodal_AUV import run_auv_inference\n"
            "except ImportError as e:\n    print('ERR', e)\n")
    env = dict(os.environ)
    env.pop("MAUV_REFERENCE_PKG", None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    assert "MAUV_REFERENCE_PKG" in r.stdout
