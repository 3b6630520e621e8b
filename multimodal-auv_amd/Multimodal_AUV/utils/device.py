"""utils/device.py surface -> mauv.device."""
from mauv.device import move_model_to_device, move_models_to_device, check_model_devices  # noqa: F401
