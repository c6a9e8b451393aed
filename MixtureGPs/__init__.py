"""Drop-in module path of the reference package ``MixtureGPs`` (MixtureGPs/__init__.py),
backed by modulatedgps_amd's MI355X kernels."""
