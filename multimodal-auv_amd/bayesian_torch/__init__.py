"""bayesian-torch 0.5.0 API names backed by mauv (the reference imports these)."""
