"""Drop-in for MixtureGPs/likelihoods.py (GaussianModified), plus the GPflow
MultiClass / RobustMax likelihood the multiclass demos build from gpflow.likelihoods."""
from modulatedgps_amd.likelihoods import GaussianModified, MultiClass, RobustMax  # noqa: F401
