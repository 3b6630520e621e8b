import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "multimodal-auv_amd")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

_LIB = os.path.join(PKG_ROOT, "mauv", "libmauv_hip.so")
if not os.path.exists(_LIB):
    # fresh checkout: the .so is git-ignored; build it (hipcc cross-compiles gfx950 on CPU)
    subprocess.run(["make", "-C", os.path.join(PKG_ROOT, "csrc"), "-j8"], check=True,
                   stdout=subprocess.DEVNULL)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
