"""Multimodal_AUV.models (mauv drop-in)."""
