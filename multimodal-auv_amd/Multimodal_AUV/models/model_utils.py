"""models/model_utils.py surface -> mauv.models."""
from mauv.layers import dnn_to_bnn  # noqa: F401
from mauv.models import (define_models, load_pretrained_resnet_as_feature_extractor,  # noqa: F401
                         load_models)
from mauv.models import ResNet50Custom, MultiModalModel, Identity  # noqa: F401
