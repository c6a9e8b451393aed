"""Drop-in for MixtureGPs/utils.py (reparameterize)."""
from modulatedgps_amd.utils import print_summary, reparameterize  # noqa: F401
