"""CPU oracle for the Multimodal-AUV hot path — TEST INFRASTRUCTURE ONLY.

This package is a plain torch-CPU fp32 restatement of the reference's hot path
(sams-tom/Multimodal-AUV @ /root/reference):

* ``resnet_ref``  — torchvision ResNet-50 v1.5 (third-party, absent from the image),
  restated with identical module names so state_dicts are interchangeable.
* ``bayes_ref``   — bayesian-torch 0.5.0 ``Conv2dReparameterization`` /
  ``LinearReparameterization`` / ``dnn_to_bnn`` (MOPED) / ``get_kl_loss``
  (third-party, pinned at ``pyproject.toml:41``, absent from the image).
* ``model_ref``   — ``ResNet50Custom`` / ``AdditiveAttention`` / ``MultiModalModel`` /
  ``define_models`` restated from ``src/Multimodal_AUV/models/base_models.py:7-90`` and
  ``models/model_utils.py:10-64``.
* ``loops_ref``   — the per-batch maths of ``train/multimodal.py:80-145``,
  ``train/unimodal.py:71-146`` and ``inference/predictors.py:54-84``.

Pinning: the restatement is checked against golden vectors produced by running the
reference's OWN Python (``MultiModalModel`` head wiring, ``train_multimodal_model``,
``evaluate_multimodal_model``, ``multimodal_predict_and_save``) with these restated
third-party layers injected (``tests/golden/make_golden.py``; fixtures in
``tests/golden/*.npz|json``).  The third-party arithmetic itself (bayesian-torch,
torchvision) is not in /root/reference and no reference test pins it, so for those
formulas parity is pinned only by the restated published algorithm.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package, and only as the checker / CPU baseline — never as the thing
measured or shipped.  The product path (``multimodal-auv_amd/mauv``) never imports it.
"""
