"""Copy one GPU check's artefacts from gpurun_out/ into profiles/<round>/ (tracked):
bench JSON line, rocprofv3 kernel stats, PMC traffic (also profiles/pmc_tendency.json, read
by bench.py) and the SQ counter means of the hot kernels.

  python tools/save_profiles.py TAG ROUND      e.g.  r01af r01
"""
import collections
import csv
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag, rnd = sys.argv[1], sys.argv[2]
g = os.path.join(ROOT, "gpurun_out")
d = os.path.join(ROOT, "profiles", rnd)
os.makedirs(d, exist_ok=True)
shutil.copy(os.path.join(g, f"bench_{tag}.json"), os.path.join(d, f"bench_{tag}.json"))
shutil.copy(os.path.join(g, f"prof_{tag}", f"{tag}_kernel_stats.csv"), os.path.join(d, f"{tag}_kernel_stats.csv"))
subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_to_json.py"), tag, "4096"], check=True,
               stdout=subprocess.DEVNULL)
shutil.copy(os.path.join(ROOT, "profiles", "pmc_tendency.json"), os.path.join(d, f"pmc_{tag}_traffic.json"))
out = {}
for name in ("sq", "sq2"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    path = os.path.join(g, f"pmc_{tag}_{name}", f"{name}_counter_collection.csv")
    if not os.path.exists(path):
        continue
    for row in csv.DictReader(open(path)):
        for k in ("tendency_kernel", "spec_passA", "spec_passB", "spec_carry", "spec_pin"):
            if k in row["Kernel_Name"]:
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, dd in acc.items():
        out.setdefault(k, {}).update({c: sum(v) / len(v) for c, v in dd.items()})
json.dump(out, open(os.path.join(d, f"pmc_{tag}_sq.json"), "w"), indent=1)
print("saved", sorted(os.listdir(d)))
