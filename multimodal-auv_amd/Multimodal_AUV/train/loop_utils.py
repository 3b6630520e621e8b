"""train/loop_utils.py surface -> mauv.loop_utils."""
from mauv.kl import get_kl_loss  # noqa: F401
from mauv.loop_utils import (define_optimizers_and_schedulers,  # noqa: F401
                             train_and_evaluate_unimodal_model,
                             train_and_evaluate_multimodal_model)
from mauv.train import (train_unimodal_model, evaluate_unimodal_model,  # noqa: F401
                        train_multimodal_model, evaluate_multimodal_model)
