"""Print the counters of tools/pmc_custom.sh passes for kernels matching a pattern
(last launch of each), e.g. python tools/pmc_show.py gpurun_out gram_x6"""
import collections
import csv
import glob
import os
import sys

root, pat = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(dict)
for d in sorted(glob.glob(os.path.join(root, "pmcc_*"))):
    f = os.path.join(d, "p_counter_collection.csv")
    if not os.path.exists(f):
        continue
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    dur = {}
    for r in csv.DictReader(open(f)):
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        name[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0][:60]
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    last = {}
    for dd in per:
        if pat in name[dd]:
            last[name[dd]] = dd
    for n, dd in last.items():
        vals[n].update(per[dd])
        vals[n]["dur_us"] = dur[dd]
for n, v in vals.items():
    print(n)
    for k, x in sorted(v.items()):
        print(f"   {k:32s} {x:14.4g}")
