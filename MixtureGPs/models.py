"""Drop-in for MixtureGPs/models.py (SGP, SMGP, SMGPModified, SVGPModified)."""
from modulatedgps_amd.models import SGP, SMGP, SMGPModified, SVGPModified  # noqa: F401
