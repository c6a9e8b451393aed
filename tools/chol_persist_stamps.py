"""Persistent K3 breakdown from in-kernel s_memtime stamps (GPU box only): builds a
-DMGP_DBG_STAMPS variant of libmgp_hip.so into var/, runs the batched Kuu Cholesky +
inverse at M (default 1024), batch 2, and prints
  chain, per step (cycles): wait for its tiles, load, L_{j+1,j} + publish, factor,
         D publish, tail;
  workers, per task (cycles, averaged over workgroups): dequeue, put, poll next,
         compute + publish, blocking wait + issue; prefetch hit rate.
Usage: python tools/chol_persist_stamps.py [M] [workers]"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
W = sys.argv[2] if len(sys.argv) > 2 else "48"
so = os.path.join(ROOT, "var", "pstamps.so")
if not os.path.exists(so) or "--rebuild" in sys.argv:
    so = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "variant_build.py"), "pstamps", "chol.hip",
                         "-DMGP_DBG_STAMPS"], check=True, capture_output=True, text=True).stdout.strip().splitlines()[-1]
os.environ["MGP_HIP_LIB"] = so
os.environ["MGP_CHOL_WORKERS"] = W
import numpy as np  # noqa: E402
import torch  # noqa: E402
from modulatedgps_amd import _lib, ops  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
Z = torch.randn(M, 8, device=dev, generator=g)
var, ls = torch.tensor([0.5], device=dev), torch.tensor([1.0], device=dev)
for _ in range(3):
    ops.kuu_potrf_trtri([Z, Z], [var, var], [ls, ls], 1e-6)
torch.cuda.synchronize()
chain = (ctypes.c_ulonglong * (2 * 128 * 8))()
work = (ctypes.c_ulonglong * (2 * 128 * 8))()
lib.mgp_dbg_persist_stamps(chain, work, 1)
ops.kuu_potrf_trtri([Z, Z], [var, var], [ls, ls], 1e-6)
torch.cuda.synchronize()
lib.mgp_dbg_persist_stamps(chain, work, 0)
c = np.array(chain, dtype=np.int64).reshape(2, 128, 8)
w = np.array(work, dtype=np.int64).reshape(2, 128, 8)
nb = (M + 63) // 64
steps = []
for j in range(nb - 1):
    t = c[0, j]
    nxt = c[0, j + 1, 0] if j + 2 < nb else t[6]
    steps.append({"wait": int(t[1] - t[0]), "load": int(t[2] - t[1]), "panel": int(t[3] - t[2]),
                  "factor": int(t[4] - t[3]), "publishD": int(t[5] - t[4]), "tail": int(t[6] - t[5]),
                  "total": int(nxt - t[0])})
tot = int(c[0, nb - 2, 6] - c[0, 0, 0])
ws = w[0, 1:int(W) + 1]
tasks = ws[:, 5].sum()
per = {k: float(ws[:, i].sum() / max(tasks, 1)) for i, k in enumerate(["dequeue", "wait_issue", "put", "poll_next",
                                                                      "compute_publish"])}
print(json.dumps({"M": M, "workers": int(W), "chain_total_cycles": tot, "chain_steps": steps,
                  "worker_per_task_cycles": per, "tasks": int(tasks),
                  "prefetch_hit_rate": float(ws[:, 6].sum() / max(tasks, 1)), "D_loads": int(ws[:, 7].sum())}))
