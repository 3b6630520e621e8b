"""Oracle: the reference's model definitions restated on torch-CPU (TEST INFRASTRUCTURE ONLY).

Follows ``src/Multimodal_AUV/models/base_models.py`` and ``models/model_utils.py``:

* ``ResNet50Custom``        base_models.py:7-29 (conv1 swapped :18, fc swapped :21)
* ``Identity``              base_models.py:31-33
* ``AdditiveAttention``     base_models.py:35-52 (``tanh(q + k)`` :48, softmax dim=1 :49,
                            ``values * weights`` with no reduction :51)
* ``MultiModalModel``       base_models.py:54-90 (fc 384->1284 :60, fc1 1284->32 :61,
                            fc2 32->C :65, no activations in the head :86-89)
* ``define_models``         model_utils.py:10-49 (three unimodal BNNs, three ImageNet-style
                            feature trunks, dnn_to_bnn over the WHOLE tri-modal model :35)
* ``load_pretrained_resnet_as_feature_extractor`` model_utils.py:52-64 (fresh 1-channel
                            conv1 :58-59, fc = Identity :60)
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .resnet_ref import resnet50, ResNet50_Weights
from .bayes_ref import dnn_to_bnn


class ResNet50Custom(nn.Module):
    def __init__(self, input_channels, num_classes):
        super().__init__()
        self.input_channels = input_channels
        self.model = resnet50(weights=ResNet50_Weights.IMAGENET1K_V1)
        self.model.conv1 = nn.Conv2d(input_channels, 64, kernel_size=7, stride=2, padding=3,
                                     bias=False)
        self.model.fc = nn.Linear(self.model.fc.in_features, num_classes)

    def forward(self, x):
        return self.model(x)

    def get_feature_size(self):
        return self.model.fc.in_features


class Identity(nn.Module):
    def forward(self, x):
        return x


class AdditiveAttention(nn.Module):
    def __init__(self, d_model, hidden_dim=128):
        super().__init__()
        self.query_projection = nn.Linear(d_model, hidden_dim)
        self.key_projection = nn.Linear(d_model, hidden_dim)
        self.value_projection = nn.Linear(d_model, hidden_dim)
        self.attention_mechanism = nn.Linear(hidden_dim, hidden_dim)

    def forward(self, query):
        keys = self.key_projection(query)
        values = self.value_projection(query)
        queries = self.query_projection(query)
        scores = torch.tanh(queries + keys)
        weights = F.softmax(self.attention_mechanism(scores), dim=1)
        return values * weights


class MultiModalModel(nn.Module):
    def __init__(self, image_model_feat, bathy_model_feat, sss_model_feat, num_classes,
                 attention_type="scaled_dot_product"):
        super().__init__()
        self.image_model_feat = image_model_feat
        self.bathy_model_feat = bathy_model_feat
        self.sss_model_feat = sss_model_feat
        self.fc = nn.Linear(384, 1284)
        self.fc1 = nn.Linear(1284, 32)
        self.fc2 = nn.Linear(32, int(num_classes))
        self.attention_type = attention_type
        self.attention_image = AdditiveAttention(2048)
        self.attention_bathy = AdditiveAttention(2048)
        self.attention_sss = AdditiveAttention(2048)

    def forward(self, inputs, bathy_tensor, sss_image):
        image_features = self.image_model_feat(inputs)
        bathy_features = self.bathy_model_feat(bathy_tensor)
        sss_features = self.sss_model_feat(sss_image)
        fi = self.attention_image(image_features)
        fb = self.attention_bathy(bathy_features)
        fs = self.attention_sss(sss_features)
        x = torch.cat([fi, fb, fs], dim=1)
        return self.fc2(self.fc1(self.fc(x)))


def load_pretrained_resnet_as_feature_extractor(input_channels=3):
    model = resnet50(weights=ResNet50_Weights.IMAGENET1K_V1)
    if input_channels == 1:
        model.conv1 = nn.Conv2d(1, 64, kernel_size=(7, 7), stride=(2, 2), padding=(3, 3),
                                bias=False)
    model.fc = Identity()
    return model


def define_models(device, num_classes, const_bnn_prior_parameters):
    image_model = ResNet50Custom(input_channels=3, num_classes=num_classes)
    bathy_model = ResNet50Custom(input_channels=3, num_classes=num_classes)
    sss_model = ResNet50Custom(input_channels=1, num_classes=num_classes)
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


DEFAULT_PRIOR = {
    "prior_mu": 0.0,
    "prior_sigma": 1.0,
    "posterior_mu_init": 0.0,
    "posterior_rho_init": -3.0,
    "type": "Reparameterization",
    "moped_enable": True,
    "moped_delta": 0.1,
}  # main.py:276-284
