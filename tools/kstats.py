"""Print the top kernels of rocprofv3 kernel_stats csv files: python tools/kstats.py FILE..."""
import csv
import sys

for f in sys.argv[1:]:
    print("==", f)
    for r in list(csv.DictReader(open(f)))[:8]:
        print(f"{float(r['AverageNs']) / 1e3:9.1f} us x{int(r['Calls']):4d}  {r['Name'][:80]}")
