"""Multimodal_AUV.train (mauv drop-in)."""
