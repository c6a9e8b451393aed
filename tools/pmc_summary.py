"""Summarise the rocprofv3 PMC passes of tools/pmc_pass.sh into per-kernel,
per-launch figures (profiles/pmc_traffic.json).

HBM traffic follows MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced
read, so bytes_read = 2 * FETCH_SIZE * 1024; bytes_written = WRITE_SIZE * 1024.
Both count L2 misses served by the Infinity Cache as well as HBM.
MFMA busy over the busy CUs: SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs * SQ_BUSY_CU_CYCLES) --
a ratio of two counts of the same shader clock, so it needs no clock.  Chip-wide
MFMA busy and the effective clock use GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs)
over the dispatch duration, which MI355X_MICROARCH.md (DVFS give-back) trusts only
for dispatches of 0.3 ms or more: on shorter ones the GUI-active window outlasts the
kernel (round 3 reported 3.2-5.1 GHz for the 6-19 us K3 launches), so below 0.3 ms
both are left out (null) and the clock-free figures stand alone.  When a pass adds
SQ_INSTS_VALU_MFMA_MOPS_F64 (units of 512 flops), the f64 MFMA count per launch is
reported too (a v_mfma_f64_16x16x4 is 2048 flops = 4 MOPS and keeps the pipe busy 64
cycles), so mfma_busy_cycles / f64_mfma_count can be checked against 64.
Usage: python tools/pmc_summary.py gpurun_out profiles/pmc_traffic.json [groups...]"""
import collections
import csv
import json
import os
import sys


def load(root, name):
    path = os.path.join(root, f"pmc_{name}", "p_counter_collection.csv")
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    names = {}
    for r in csv.DictReader(open(path)):
        key = r["Dispatch_Id"]
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        names[key] = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
    return per, dur, names


def kernel_key(name):
    """Kernel base name; the split-f16 instances of K1/K4/K5 (template flags
    `true`) are kept apart from their split-bf16 instances."""
    base = name.split("::")[-1].split("<")[0]
    args = name.split("<", 1)[1] if "<" in name else ""
    flags = [a.strip() for a in args.split(">")[0].split(",")]
    if base == "trsm_stats_x6_kernel" and flags[1:] == ["true", "true", "true"]:
        return "trsm_stats_f16x8_kernel"        # split-f16 in and out, + the A image's e4m3 plane
    if base == "trsm_stats_x6_kernel" and flags[1:3] == ["true", "true"]:
        return "trsm_stats_f16_kernel"          # split-f16 images in and out
    if base == "trsm_stats_x6_kernel" and flags[1:2] == ["true"]:
        return "trsm_stats_x6f16_kernel"        # split-bf16 in, split-f16 A image out
    if base == "gram_x6_kernel" and flags[2:3] == ["true"]:
        return "gram_f16_kernel"
    if base == "grad_a_s_kernel" and flags[:1] == ["true"]:
        return "grad_a_s_f16_kernel"
    if base == "expert_cond_x6_kernel" and flags[1:3] == ["true", "true"]:
        return "expert_cond_f16x8_kernel"       # split-f16 hi products + e4m3 cross terms
    if base == "expert_cond_x6_kernel" and flags[1:4] == ["true", "false", "true"]:
        return "expert_cond_f16c_kernel"        # split-f16, also writing the C_k images (training)
    if base == "expert_cond16_kernel" and flags[:1] == ["true"]:
        return "expert_cond16c_kernel"          # 16x16x32, also writing the C_k images (training)
    if base == "expert_cond16_pair_kernel" and flags[:1] == ["true"]:
        return "expert_cond16c_pair_kernel"     # both layers in one launch, with the C_k images
    if base in ("expert_cond_x6_kernel", "rbf_kuf_x6_kernel") and "true" in flags:
        return base.replace("_x6_", "_f16_")
    return base


MIN_CLOCK_DISPATCH_S = 0.3e-3


def main(root, out, groups=("SQ_WAVE_CYCLES", "FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum")):
    res = collections.defaultdict(lambda: collections.defaultdict(list))
    for group in groups:
        if not os.path.exists(os.path.join(root, f"pmc_{group}", "p_counter_collection.csv")):
            continue
        per, dur, names = load(root, group)
        for d, cs in per.items():
            if "mgp::" not in names[d]:
                continue
            k = kernel_key(names[d])
            for c, v in cs.items():
                res[k][c].append(v)
            res[k]["duration_s"].append(dur[d])
    summary = {}
    for k, cs in res.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"launches_sampled": len(cs.get("FETCH_SIZE", []))}
        if avg["duration_s"] > 0:  # PMC-mode timestamps are zero for some dispatches (durations: kernel-trace stats)
            e["avg_duration_us"] = avg["duration_s"] * 1e6
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            rd = 2.0 * avg["FETCH_SIZE"] * 1024
            wr = avg["WRITE_SIZE"] * 1024
            e.update(hbm_read_bytes=rd, hbm_write_bytes=wr, hbm_bytes_per_launch=rd + wr)
        if "TCC_HIT_sum" in avg:
            e["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"], 1.0)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            e["mfma_busy_cycles"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"]
            if avg.get("SQ_BUSY_CU_CYCLES"):
                # MFMA busy over the CUs that had waves resident (latency-bound
                # kernels such as the K3 chain occupy a few CUs of the 256); clock-free
                e["mfma_busy_active_cus"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (4.0 * avg["SQ_BUSY_CU_CYCLES"])
            long_enough = avg.get("duration_s", 0.0) >= MIN_CLOCK_DISPATCH_S
            if avg.get("GRBM_GUI_ACTIVE") and long_enough:
                cyc = avg["GRBM_GUI_ACTIVE"] / 8.0
                e["mfma_busy"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc)
                e["effective_clock_ghz"] = cyc / (avg["duration_s"] * 1e9)
                if avg.get("SQ_BUSY_CU_CYCLES"):
                    e["active_cu_fraction"] = avg["SQ_BUSY_CU_CYCLES"] / (256.0 * cyc)
            else:
                e["effective_clock_ghz"] = None
                e["clock_note"] = "dispatch < 0.3 ms: GRBM_GUI_ACTIVE outlasts the kernel, no clock derived"
        if avg.get("SQ_WAVE_CYCLES"):   # wave-cycle buckets (issuing / waiting on a dependency or pipe / parked)
            wc = avg["SQ_WAVE_CYCLES"]
            e["wave_cycles_issuing"] = avg.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
            e["wave_cycles_wait_inst"] = avg.get("SQ_WAIT_INST_ANY", 0.0) / wc
            e["wave_cycles_wait_any"] = avg.get("SQ_WAIT_ANY", 0.0) / wc
        if avg.get("SQ_INSTS_LDS"):
            e["lds_bank_conflict_cycles_per_lds_inst"] = avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / avg["SQ_INSTS_LDS"]
        if "SQ_INSTS_VALU_MFMA_MOPS_F64" in avg:
            e["f64_mfma_count"] = avg["SQ_INSTS_VALU_MFMA_MOPS_F64"] / 4.0
            if e.get("mfma_busy_cycles") and e["f64_mfma_count"] > 0:
                e["mfma_busy_cycles_per_f64_mfma"] = e["mfma_busy_cycles"] / e["f64_mfma_count"]
        summary[k] = e
    json.dump({"source": os.environ.get("PMC_SOURCE", "rocprofv3 --pmc passes of tools/pmc_pass.sh (tools/bench_kernels.py, c3)"),
               "corrections": "bytes_read = 2 * FETCH_SIZE KiB (gfx950 wide-read undercount), "
                              "bytes_written = WRITE_SIZE KiB",
               "kernels": summary}, open(out, "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 3:
        main(sys.argv[1], sys.argv[2], tuple(sys.argv[3:]))
    else:
        main(sys.argv[1], sys.argv[2])
