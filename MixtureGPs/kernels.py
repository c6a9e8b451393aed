"""Stand-in for gpflow.kernels.SquaredExponential as used by the demos (demo_tf2.py:37-38)."""
from modulatedgps_amd.kernels import SquaredExponential  # noqa: F401
