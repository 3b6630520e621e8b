"""train/multimodal.py surface -> mauv.train (batched MC, fused KL / CE / NaN guard)."""
import sys

import mauv.train as _impl
from mauv.kl import get_kl_loss  # noqa: F401  (patchable, as in the reference)
from mauv.checkpointing import save_model  # noqa: F401
from ._patchable import call_with_module_kl


def train_multimodal_model(*args, **kwargs):
    return call_with_module_kl(sys.modules[__name__], _impl.train_multimodal_model, *args,
                               **kwargs)


def evaluate_multimodal_model(*args, **kwargs):
    return call_with_module_kl(sys.modules[__name__], _impl.evaluate_multimodal_model, *args,
                               **kwargs)
