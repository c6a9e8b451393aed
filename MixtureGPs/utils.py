"""Drop-in for MixtureGPs/utils.py (reparameterize)."""
from modulatedgps_amd.utils import reparameterize  # noqa: F401
