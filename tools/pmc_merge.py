"""Merge the kernels of a tools/pmc_summary.py output into profiles/pmc_traffic.json
(entries of the same kernel are replaced).  Usage: python tools/pmc_merge.py SUMMARY.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
d = json.load(open(path))
new = json.load(open(sys.argv[1]))["kernels"]
d["kernels"].update(new)
json.dump(d, open(path, "w"), indent=1)
print("merged", sorted(new))
