"""tf.data replacement for the demos' minibatch pipeline (see modulatedgps_amd.data)."""
from modulatedgps_amd.data import Dataset  # noqa: F401
