"""train/checkpointing.py surface -> mauv.checkpointing."""
from mauv.checkpointing import save_model, load_and_fix_state_dict, remap_keys  # noqa: F401
