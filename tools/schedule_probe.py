"""A/B of the ELBO step's launch schedules (modulatedgps_amd.config.STEP_SCHEDULES)
at BASELINE c3: ms per step (HIP-synchronised wall blocks, no events inside) and the
in-step K3 stage (event brackets, separate block), interleaved rounds; the ELBO with
a fixed Philox key must be bit-identical across schedules.
Usage (GPU box): python tools/schedule_probe.py [rounds]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from modulatedgps_amd import config  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    scheds = sys.argv[2].split(",") if len(sys.argv) > 2 else list(config.STEP_SCHEDULES)
    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS["c3"]
    X_np, Y_np, layers = bench.synthetic(cfg, 0, dev)
    model = bench.build_model(cfg, layers, dev, num_data=cfg[0])
    X = torch.from_numpy(X_np).to(dev)
    Y = torch.from_numpy(Y_np).to(dev)
    res = {s: {"ms": [], "k3_us": [], "elbo": None} for s in scheds}
    for r in range(rounds):
        for s in scheds:
            config.set_step_schedule(s)
            for _ in range(5):
                model._build_likelihood(X, Y)
            torch.cuda.synchronize()
            e = float(model._build_likelihood(X, Y, seed=777).item())
            if res[s]["elbo"] is None:
                res[s]["elbo"] = e
            t0 = time.perf_counter()
            for _ in range(40):
                model._build_likelihood(X, Y)
            torch.cuda.synchronize()
            res[s]["ms"].append((time.perf_counter() - t0) / 40 * 1e3)
            timing = {}
            for _ in range(10):
                model._build_likelihood(X, Y, timing=timing)
            torch.cuda.synchronize()
            st = bench.stage_stats(timing)
            res[s]["k3_us"].append(st["kuu_chol"][0] * 1e3)
            print(json.dumps({"round": r, "sched": s, "ms": round(res[s]["ms"][-1], 4),
                              "k3_us": round(res[s]["k3_us"][-1], 1)}), flush=True)
    out = {s: {"ms_median": float(np.median(v["ms"])), "k3_us_median": float(np.median(v["k3_us"])),
               "elbo_fixed_key": v["elbo"]} for s, v in res.items()}
    ref = out[scheds[0]]["elbo_fixed_key"]
    out["bit_identical"] = all(v["elbo_fixed_key"] == ref for v in out.values() if isinstance(v, dict))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
