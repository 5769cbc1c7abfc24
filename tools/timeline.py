"""Print a per-step kernel timeline from a rocprofv3 kernel_trace.csv.
usage: python tools/timeline.py TRACE.csv [first_kernel_substring] [nsteps] [MEMORY_COPY_TRACE.csv]
(the memory-copy trace's copies are merged in as "COPY <direction>" rows)"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
key = sys.argv[2] if len(sys.argv) > 2 else "tendency_kernel"
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
if len(sys.argv) > 4:
    for r in csv.DictReader(open(sys.argv[4])):
        r = dict(r)
        r["Kernel_Name"] = f"COPY {r.get('Direction', '?')} {r.get('Bytes', r.get('Size', ''))}"
        r.setdefault("Queue_Id", "cp")
        rows.append(r)
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [k for k, r in enumerate(rows) if key in r["Kernel_Name"]]
# the last nsteps+1 occurrences delimit nsteps steps
sel = starts[-(nsteps + 1):]
for a, b in zip(sel[:-1], sel[1:]):
    t0 = int(rows[a]["Start_Timestamp"])
    print("---- step")
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{r.get('Queue_Id', '?'):>3} {r['Kernel_Name'][:70]}")
