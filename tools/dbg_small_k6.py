"""Debug: K6 backward (tests/test_gpu_backward.py::test_elbo_terms_backward) at tiny N."""
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_backward import test_elbo_terms_backward  # noqa: E402

dev = torch.device("cuda", 0)
for args in [(2, 1, 1, 1, 0.5, 1, False), (3, 1, 1, 1, 0.5, 1, False), (8, 1, 1, 1, 0.5, 1, False),
             (2, 2, 1, 1, 0.5, 1, False), (2, 1, 1, 1, 0.5, 3, False), (5, 2, 3, 1, 0.5, 2, True), (16, 2, 1, 1, 0.5, 1, False),
             (17, 2, 1, 1, 0.5, 1, False), (33, 2, 1, 1, 0.5, 1, False)]:
    try:
        test_elbo_terms_backward(dev, *args)
        print(args, "ok", flush=True)
    except AssertionError as e:
        print(args, "FAIL", str(e).split("\n")[0][:200], flush=True)
    except Exception:
        print(args, "ERROR", traceback.format_exc()[-300:], flush=True)
