"""Build libmgp_hip.so (gfx950) in-tree with hipcc.

    python -m modulatedgps_amd.build [-v]

The shared library has a plain C ABI (include/mgp_hip.h) and no torch
dependency; it links only the HIP runtime.  Objects are compiled in parallel
and the library is relinked only when a source or header is newer.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(PKG, "_build")
LIB = os.path.join(PKG, "libmgp_hip.so")
ARCH = os.environ.get("MGP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CXXFLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-I", INCLUDE, "-I", CSRC,
            "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


# per-source flags: chol.hip's step launches take their hot scalar arguments first, and the
# dispatch preloads up to 16 argument dwords into SGPRs (gfx950 kernel-argument preload),
# so a K3 step's first tile loads wait for no kernel-argument fetch
FILE_FLAGS = {"chol.hip": ["-mllvm", "-amdgpu-kernarg-preload-count=16"]}


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    hs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    return hs


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _compile(src, hdr_time, verbose, extra):
    obj = os.path.join(BUILD, os.path.basename(src).replace(".hip", ".o"))
    if _mtime(obj) >= max(_mtime(src), hdr_time) and not extra:
        return obj
    cmd = [HIPCC, *CXXFLAGS, *FILE_FLAGS.get(os.path.basename(src), []), *extra, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, flush=True)
    return obj


def build(verbose=False, extra_flags=()):
    """Compile every csrc/*.hip for gfx950 and link modulatedgps_amd/libmgp_hip.so."""
    os.makedirs(BUILD, exist_ok=True)
    srcs = _sources()
    hdr_time = max([_mtime(h) for h in _headers()] + [0.0])
    extra = list(extra_flags)
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr_time, verbose, extra), srcs))
    if _mtime(LIB) < max(_mtime(o) for o in objs) or extra:
        tmp = LIB + ".tmp"
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
    return LIB


ASAN_BUILD = os.path.join(PKG, "_build_asan")
ASAN_LIB = os.path.join(ASAN_BUILD, "libmgp_hip_asan.so")


def asan_runtime():
    """The clang AddressSanitizer runtime the host-ASan library links against (preloaded
    into the Python process that loads it), or None."""
    base = "/opt/rocm/lib/llvm/lib/clang"
    if not os.path.isdir(base):
        return None
    for v in sorted(os.listdir(base), reverse=True):
        p = os.path.join(base, v, "lib", "linux", "libclang_rt.asan-x86_64.so")
        if os.path.exists(p):
            return p
    return None


def build_asan(verbose=False):
    """libmgp_hip.so with its HOST code built under AddressSanitizer (-Xarch_host
    -fsanitize=address; the gfx950 device code is the same, GPU sanitizers are not used) into
    modulatedgps_amd/_build_asan/ -- for the CPU tests of the C-ABI's host paths
    (tests/test_host_asan.py).  Not the product library."""
    os.makedirs(ASAN_BUILD, exist_ok=True)
    srcs = _sources()
    hdr_time = max([_mtime(h) for h in _headers()] + [0.0])
    flags = ["-O1", "-g", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-I", INCLUDE, "-I", CSRC,
             "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]

    def one(src):
        obj = os.path.join(ASAN_BUILD, os.path.basename(src).replace(".hip", ".o"))
        if _mtime(obj) >= max(_mtime(src), hdr_time):
            return obj
        cmd = [HIPCC, *flags, *FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc (asan) failed for {src}:\n{r.stdout}\n{r.stderr}")
        return obj
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(one, srcs))
    if _mtime(ASAN_LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-fsanitize=address", "-shared-libasan",
               "-o", ASAN_LIB + ".tmp", *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link (asan) failed:\n{r.stdout}\n{r.stderr}")
        os.replace(ASAN_LIB + ".tmp", ASAN_LIB)
    return ASAN_LIB


C_ABI_SRC = os.path.join(ROOT, "tests", "c_abi", "elbo_c.cpp")
C_ABI_BIN = os.path.join(ROOT, "tests", "c_abi", "elbo_c")


def build_c_abi_test(verbose=False):
    """tests/c_abi/elbo_c: a host program that runs one ELBO through the C-ABI of
    libmgp_hip.so alone (no torch), for tests/test_gpu_c_abi.py.  Linked against the
    in-tree library by a relative rpath, so it runs from the snapshot on the GPU box."""
    lib = build(verbose)
    if _mtime(C_ABI_BIN) >= max(_mtime(C_ABI_SRC), _mtime(lib), _mtime(os.path.join(INCLUDE, "mgp_hip.h"))):
        return C_ABI_BIN
    cmd = [HIPCC, "-O2", "-std=c++17", "-I", INCLUDE, C_ABI_SRC, "-o", C_ABI_BIN, "-L", PKG, "-lmgp_hip",
           "-Wl,-rpath,$ORIGIN/../../modulatedgps_amd"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"C-ABI test program failed to build:\n{r.stdout}\n{r.stderr}")
    return C_ABI_BIN


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
    print(build_c_abi_test(verbose="-v" in sys.argv))
