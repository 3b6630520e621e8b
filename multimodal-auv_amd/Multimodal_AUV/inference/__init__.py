"""Multimodal_AUV.inference (mauv drop-in)."""
