"""Route a drop-in module's (possibly monkey-patched) ``get_kl_loss`` into mauv.train.

The reference's tests patch ``Multimodal_AUV.train.multimodal.get_kl_loss`` /
``...unimodal.get_kl_loss`` (unittests/test_train.py:227,536); the loops here honour that.
"""
import mauv.train as impl


def call_with_module_kl(module, fn, *args, **kwargs):
    saved = impl.get_kl_loss
    impl.get_kl_loss = module.get_kl_loss
    try:
        return fn(*args, **kwargs)
    finally:
        impl.get_kl_loss = saved
