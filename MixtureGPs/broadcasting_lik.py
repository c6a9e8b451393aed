"""Drop-in for MixtureGPs/broadcasting_lik.py (BroadcastingLikelihood)."""
from modulatedgps_amd.broadcasting_lik import BroadcastingLikelihood  # noqa: F401
