"""modulatedgps_amd: MI355X-native (gfx950) SMGP ELBO hot path of LouieMiddle/ModulatedGPs.

Host side in Python on PyTorch-ROCm (device memory, streams, torch.distributed);
all arithmetic in hand-written HIP kernels of libmgp_hip.so behind the C-ABI of
include/mgp_hip.h.  The drop-in reference API lives under the ``MixtureGPs``
package at the repository root (same module paths as the reference).
"""
from . import _lib
from ._lib import MGPError, MGPLibraryError, MGPLinAlgError

__version__ = "0.1.0"


def library():
    """Load (and return) libmgp_hip.so; raises MGPLibraryError if it is missing."""
    return _lib.load()
