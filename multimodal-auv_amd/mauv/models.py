"""The reference's model surface (models/base_models.py, models/model_utils.py) on the HIP engine.

Same classes, constructor signatures, attribute names and state_dict keys as the reference:

* ``ResNet50Custom(input_channels, num_classes)``        base_models.py:7-29
* ``Identity``                                          base_models.py:31-33
* ``AdditiveAttention(d_model, hidden_dim=128)``         base_models.py:35-52
* ``MultiModalModel(img, bathy, sss, num_classes, attention_type=...)`` base_models.py:54-90
* ``define_models(device, num_classes, const_bnn_prior_parameters)``   model_utils.py:10-49
* ``load_pretrained_resnet_as_feature_extractor(input_channels=3)``    model_utils.py:52-64
* ``load_models(model_paths, device, num_classes)``                    model_utils.py:66-101

Additions (not in the reference): ``mc_forward(..., num_mc)`` on the trunk / tri-modal model
returns all MC samples ``[num_mc, B, C]`` from one batched launch per layer; the loops in
``mauv.train`` / ``mauv.predict`` use it.  ``forward`` keeps the reference's one-sample contract.
"""
import logging
import os

import torch
import torch.nn as nn

from . import engine
from .layers import dnn_to_bnn, is_bayesian
from .resnet import resnet50, ResNet


class ResNet50Custom(nn.Module):
    def __init__(self, input_channels, num_classes):
        super().__init__()
        self.input_channels = input_channels
        self.model = resnet50(weights="IMAGENET1K_V1")
        self.model.conv1 = nn.Conv2d(input_channels, 64, kernel_size=7, stride=2, padding=3,
                                     bias=False)
        self.model.fc = nn.Linear(self.model.fc.in_features, num_classes)

    def forward(self, x):
        return self.mc_forward(x, 1)[0]

    def mc_forward(self, x, num_mc):
        # this wrapper is the engine root (same root as get_kl_loss(self) / the optimiser)
        return engine.run_trunk_mc(self.model, x, num_mc, state=engine.root_state(self))

    def get_feature_size(self):
        return self.model.fc.in_features


class Identity(nn.Module):
    def forward(self, x):
        return x


class AdditiveAttention(nn.Module):
    """base_models.py:35-52.  Inside MultiModalModel its maths runs fused in the head schedule
    (engine.HeadRunner); called on its own, ``forward`` runs one stochastic pass through the
    same kernels: q|k|v as ONE GEMM over [Wq;Wk;Wv], tanh(q + k), Wm, softmax over the
    hidden dim, v * a (differentiable)."""

    def __init__(self, d_model, hidden_dim=128):
        super().__init__()
        self.query_projection = nn.Linear(d_model, hidden_dim)
        self.key_projection = nn.Linear(d_model, hidden_dim)
        self.value_projection = nn.Linear(d_model, hidden_dim)
        self.attention_mechanism = nn.Linear(hidden_dim, hidden_dim)

    def forward(self, query):
        return self.mc_forward(query, 1)[0]

    def mc_forward(self, query, num_mc):
        if not is_bayesian(self.query_projection):
            raise TypeError("AdditiveAttention must be converted with dnn_to_bnn "
                            "(models/model_utils.py:35) before running")
        return engine.run_attention_mc(self, query, num_mc)


class MultiModalModel(nn.Module):
    def __init__(self, image_model_feat, bathy_model_feat, sss_model_feat, num_classes,
                 attention_type="scaled_dot_product"):
        super().__init__()
        self.image_model_feat = image_model_feat
        self.bathy_model_feat = bathy_model_feat
        self.sss_model_feat = sss_model_feat
        self.fc = nn.Linear(384, 1284)
        self.fc1 = nn.Linear(1284, 32)
        num_classes = int(num_classes)
        if not isinstance(num_classes, int):
            raise TypeError("num_classes must be an integer")
        self.fc2 = nn.Linear(32, num_classes)
        self.attention_type = attention_type
        self.attention_image = AdditiveAttention(2048)
        self.attention_bathy = AdditiveAttention(2048)
        self.attention_sss = AdditiveAttention(2048)

    def forward(self, inputs, bathy_tensor, sss_image):
        """One stochastic forward pass -> logits [B, C] (base_models.py:74-90)."""
        return self.mc_forward(inputs, bathy_tensor, sss_image, 1)[0]

    def mc_forward(self, inputs, bathy_tensor, sss_image, num_mc):
        """``num_mc`` stochastic forward passes in one batched launch -> [num_mc, B, C]."""
        if not is_bayesian(self.fc):
            raise TypeError("MultiModalModel must be converted with dnn_to_bnn "
                            "(models/model_utils.py:35) before running")
        return engine.run_multimodal_mc(self, inputs, bathy_tensor, sss_image, num_mc)


def load_pretrained_resnet_as_feature_extractor(input_channels: int = 3) -> nn.Module:
    """ImageNet-architecture trunk with fc = Identity; 1-channel variant gets a fresh conv1.
    (ImageNet weights cannot be downloaded offline: synthetic torchvision-style init.)"""
    model = resnet50(weights="IMAGENET1K_V1")
    if input_channels == 1:
        model.conv1 = nn.Conv2d(1, 64, kernel_size=(7, 7), stride=(2, 2), padding=(3, 3),
                                bias=False)
    model.fc = Identity()
    return model


def define_models(device, num_classes, const_bnn_prior_parameters):
    """models/model_utils.py:10-49 — same construction order, same dict keys."""
    try:
        image_model = ResNet50Custom(input_channels=3, num_classes=num_classes)
        bathy_model = ResNet50Custom(input_channels=3, num_classes=num_classes)
        sss_model = ResNet50Custom(input_channels=1, num_classes=num_classes)
        logging.info("Loading pretrained models as feature extractors.")
        logging.info("Converting models to Bayesian versions.")
        dnn_to_bnn(image_model, const_bnn_prior_parameters)
        dnn_to_bnn(bathy_model, const_bnn_prior_parameters)
        dnn_to_bnn(sss_model, const_bnn_prior_parameters)
        image_model_feat = load_pretrained_resnet_as_feature_extractor()
        bathy_model_feat = load_pretrained_resnet_as_feature_extractor()
        sss_model_feat = load_pretrained_resnet_as_feature_extractor(input_channels=1)
        multimodal_model = MultiModalModel(image_model_feat, bathy_model_feat, sss_model_feat,
                                           num_classes)
        dnn_to_bnn(multimodal_model, const_bnn_prior_parameters)
        return {
            "image_model": image_model,
            "bathy_model": bathy_model,
            "sss_model": sss_model,
            "multimodal_model": multimodal_model,
            "image_model_feat": image_model_feat,
            "bathy_model_feat": bathy_model_feat,
            "sss_model_feat": sss_model_feat,
        }
    except Exception as e:
        logging.error(f"Error defining models: {e}", exc_info=True)
        raise


def load_models(model_paths, device, num_classes):
    """models/model_utils.py:66-101 (plain trunks, optional per-modality state_dicts)."""
    image_model_feat = load_pretrained_resnet_as_feature_extractor()
    channels_model_feat = load_pretrained_resnet_as_feature_extractor()
    sss_model_feat = load_pretrained_resnet_as_feature_extractor(input_channels=1)
    loaded = {"image": image_model_feat, "channels": channels_model_feat, "sss": sss_model_feat}
    for key, model in loaded.items():
        path = model_paths.get(key)
        try:
            if path and os.path.exists(path):
                model.load_state_dict(torch.load(path, map_location=device, weights_only=True))
                logging.info(f"{key.capitalize()} model loaded successfully from {path}.")
            else:
                logging.warning(f"Path not found for model: {key} -> {path}")
        except Exception as inner_e:
            logging.error(f"Failed to load {key} model from {path}: {inner_e}", exc_info=True)
    return image_model_feat, channels_model_feat, sss_model_feat


DEFAULT_PRIOR = {
    "prior_mu": 0.0,
    "prior_sigma": 1.0,
    "posterior_mu_init": 0.0,
    "posterior_rho_init": -3.0,
    "type": "Reparameterization",
    "moped_enable": True,
    "moped_delta": 0.1,
}  # main.py:276-284
