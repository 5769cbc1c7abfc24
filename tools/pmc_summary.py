"""Per-kernel means of every counter in the rocprofv3 --pmc passes of tools/pmc.sh TAG
(grouped by the kernel's template name; FETCH_SIZE reported x2 in bytes, WRITE_SIZE in
bytes, per MI355X_MICROARCH.md's gfx950 correction).  usage: python tools/pmc_summary.py TAG [skip]"""
import collections
import csv
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("qg::", "")


def main():
    tag = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{tag}_*", "*_counter_collection.csv")):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                per[(k, row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
        bykern = collections.defaultdict(list)
        for (k, d), cs in per.items():
            bykern[k].append((int(d), cs))
        for k, lst in bykern.items():
            lst.sort()
            for _, cs in lst[skip:] if len(lst) > skip else lst:
                for c, v in cs.items():
                    acc[k][c].append(v)
    for k in sorted(acc):
        if not any(s in k for s in ("spec_", "tendency", "slot_move", "pcg")):
            continue
        print(k)
        for c in sorted(acc[k]):
            v = acc[k][c]
            m = sum(v) / len(v)
            if c == "FETCH_SIZE":
                print(f"   {c:26s} {2 * m * 1024 / 1e6:12.1f} MB (x2)  n={len(v)}")
            elif c == "WRITE_SIZE":
                print(f"   {c:26s} {m * 1024 / 1e6:12.1f} MB        n={len(v)}")
            else:
                print(f"   {c:26s} {m:14.4g}  n={len(v)}")


if __name__ == "__main__":
    main()
