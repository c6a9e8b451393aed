"""Host-side AddressSanitizer run of the C-ABI boundary (the sanitizer plan: GPU
sanitizers are not available on this pool, so only the host code is instrumented).

The library is rebuilt with its host code under -fsanitize=address (modulatedgps_amd.build
.build_asan; the gfx950 device code is unchanged) and every entry of include/mgp_hip.h is
called in a child process, with the clang ASan runtime preloaded, under three argument
patterns (tests/asan_probe.py): zero sizes, null pointers, and pointers into a zeroed host
buffer.  CPU only -- without a GPU each entry either rejects its arguments or returns the
error of its first HIP call; the test fails on any AddressSanitizer report or crash (an
argument check that reads through a pointer it has not validated, a host-array overrun)."""
import os
import subprocess
import sys

import pytest

from modulatedgps_amd import _lib, build as B

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def asan_lib():
    rt = B.asan_runtime()
    if rt is None:
        pytest.skip("clang AddressSanitizer runtime not found under /opt/rocm/lib/llvm")
    return B.build_asan(), rt


@pytest.mark.parametrize("pattern", ["zero", "null", "buf"])
def test_c_abi_entries_clean_under_host_asan(asan_lib, pattern):
    lib, rt = asan_lib
    env = dict(os.environ, MGP_HIP_LIB=lib, LD_PRELOAD=rt,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=86")
    r = subprocess.run([sys.executable, os.path.join(HERE, "asan_probe.py"), pattern], env=env,
                       capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    n = len([s for s in _lib.SIGNATURES if s not in ("mgp_dbg_chol_stamps", "mgp_dbg_k4_stamps")])
    assert "asan runtime True" in r.stdout   # the sanitizer is really in the process
    assert f"entries {n}" in r.stdout
