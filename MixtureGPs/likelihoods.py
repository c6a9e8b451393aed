"""Drop-in for MixtureGPs/likelihoods.py (GaussianModified)."""
from modulatedgps_amd.likelihoods import GaussianModified  # noqa: F401
