"""Driver for tests/test_host_asan.py (run in a child process with the AddressSanitizer
runtime preloaded and MGP_HIP_LIB pointing at the host-ASan library): calls every entry of
the C-ABI binding table once per argument pattern and prints each status.
    zero: null pointers, zero sizes          null: null pointers, sizes 16
    buf:  every pointer at one zeroed 1 MiB host buffer, sizes 16
Without a GPU, an entry that gets past its argument checks returns the HIP error of its
first runtime call; what the test asserts is that none touches host memory it must not."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulatedgps_amd import _lib  # noqa: E402

SKIP = {"mgp_dbg_chol_stamps", "mgp_dbg_k4_stamps"}   # debug stamp readers (copy a fixed table)


def main(pattern):
    lib = _lib.load()
    print("asan runtime", hasattr(ctypes.CDLL(None), "__asan_init"), flush=True)
    buf = ctypes.create_string_buffer(1 << 20)
    n = 0
    for name, (_, args) in sorted(_lib.SIGNATURES.items()):
        if name in SKIP:
            continue
        vals = []
        for a in args:
            if a is ctypes.c_void_p:
                vals.append(ctypes.addressof(buf) if pattern == "buf" else None)
            elif a in (ctypes.c_float, ctypes.c_double):
                vals.append(1.0)
            else:
                vals.append(0 if pattern == "zero" else 16)
        r = getattr(lib, name)(*vals)
        print(name, r, flush=True)
        n += 1
    print("entries", n, flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
