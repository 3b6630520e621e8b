"""bayesian_torch.models (mauv-backed)."""
