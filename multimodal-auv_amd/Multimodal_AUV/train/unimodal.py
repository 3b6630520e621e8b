"""train/unimodal.py surface -> mauv.train."""
import sys

import mauv.train as _impl
from mauv.kl import get_kl_loss  # noqa: F401  (patchable, as in the reference)
from mauv.checkpointing import save_model  # noqa: F401
from ._patchable import call_with_module_kl


def train_unimodal_model(*args, **kwargs):
    return call_with_module_kl(sys.modules[__name__], _impl.train_unimodal_model, *args, **kwargs)


def evaluate_unimodal_model(*args, **kwargs):
    return call_with_module_kl(sys.modules[__name__], _impl.evaluate_unimodal_model, *args,
                               **kwargs)
