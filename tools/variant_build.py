"""Build a variant of libmgp_hip.so with extra -D flags on one source, for A/B timing
on the GPU box via MGP_HIP_LIB (the in-tree library is left alone).
    python tools/variant_build.py NAME split3.hip -DFOO=1 ...   -> abvar/NAME.so (travels to the box)"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulatedgps_amd import build as B  # noqa: E402

name, src, flags = sys.argv[1], sys.argv[2], sys.argv[3:]
B.build()
out_dir = os.path.join(B.ROOT, "abvar")
os.makedirs(out_dir, exist_ok=True)
obj = os.path.join(out_dir, name + "_" + src.replace(".hip", ".o"))
subprocess.run([B.HIPCC, *B.CXXFLAGS, *B.FILE_FLAGS.get(src, []), *flags, "-c", os.path.join(B.CSRC, src), "-o", obj], check=True)
objs = [os.path.join(B.BUILD, f) for f in sorted(os.listdir(B.BUILD))
        if f.endswith(".o") and f != src.replace(".hip", ".o")]
subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", os.path.join(out_dir, name + ".so"),
                obj, *objs], check=True)
os.remove(obj)
print(os.path.join(out_dir, name + ".so"))
