"""One ELBO step's kernel timeline from a rocprofv3 kernel trace (bench.py run
under `rocprofv3 --kernel-trace`): start / end / duration (us, relative to the
step's chol_prep) and queue of every dispatch between two chol_prep launches;
the K3 step launches are summarised on one line (with --steps: one line per launch,
its duration and the gap to the previous launch).
Usage: python tools/timeline.py gpurun_out/prof/bench_kernel_trace.csv [step index] [--steps]"""
import csv
import sys


def main(path, which=60, per_step=False):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "chol_prep" in r["Kernel_Name"]]
    i0, i1 = idx[which], idx[which + 1]
    t0 = int(rows[i0]["Start_Timestamp"])
    steps = []
    for r in rows[i0:i1 + 1]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:64]
        if "chol_step" in name:
            if per_step:
                gap = s - steps[-1][1] if steps else 0.0
                print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  gap {gap:5.1f}  q={r['Queue_Id']} {name}")
            steps.append((s, e))
            continue
        print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  q={r['Queue_Id']} {name}")
    if steps:
        print(f"chol_step x{len(steps)}: {steps[0][0]:.1f} .. {steps[-1][1]:.1f} us")
    print(f"step: {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--steps"]
    main(args[0], int(args[1]) if len(args) > 1 else 60, "--steps" in sys.argv)
