"""Multimodal_AUV.utils (mauv drop-in)."""
