"""MFMA busy of the K3 kernels from tools/k3_pair_probe.sh's SQ passes
(gpurun_out/k3pmc{1,0}: tile pairs / one tile per workgroup).
Usage: python tools/k3_pmc_show.py [gpurun_out]"""
import collections
import csv
import json
import os
import sys


def summary(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names, dur = {}, {}
    for r in csv.DictReader(open(path)):
        k = r["Dispatch_Id"]
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        names[k] = r["Kernel_Name"].split("(")[0].split("::")[-1]
        dur[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for k, d in per.items():
        n = names[k]
        if not n.startswith("chol_"):
            continue
        for c, x in d.items():
            agg[n][c] += x
        agg[n]["dur"] += dur[k]
        agg[n]["launches"] += 1
    out = {}
    for n, d in agg.items():
        cyc = d["GRBM_GUI_ACTIVE"] / 8.0
        out[n] = {"launches": int(d["launches"]), "avg_us": round(d["dur"] / d["launches"] * 1e6, 2),
                  "mfma_busy_active_cus": round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (4.0 * d["SQ_BUSY_CU_CYCLES"]), 3),
                  "mfma_busy": round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc), 3),
                  "active_cu_fraction": round(d["SQ_BUSY_CU_CYCLES"] / (256.0 * cyc), 3)}
    return out


def main(root):
    res = {}
    for v, name in (("1", "pairs (default)"), ("0", "tiles (MGP_CHOL_PAIR=0)")):
        p = os.path.join(root, f"k3pmc{v}", "pmc_SQ_WAVE_CYCLES", "p_counter_collection.csv")
        if os.path.exists(p):
            res[name] = summary(p)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
