"""Reduce the FETCH_SIZE / WRITE_SIZE passes of tools/pmc.sh to per-launch HBM bytes of the
hot kernels, written to profiles/pmc_tendency.json (read by bench.py for roofline.traffic).

  python tools/pmc_to_json.py TAG N  [out.json]

Corrections (MI355X_MICROARCH.md, HBM / rocprofv3 section): counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a coalesced streaming read, so it is doubled; WRITE_SIZE
is taken as is.  The kernels here load 8 B per lane (not the guide's calibrated 16 B); the
doubled figure agrees with the algorithmic read bytes of the tendency kernel to ~6 %, which
is the calibration we rely on (Measurement)."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"tendency": "tendency_kernel", "passA": "spec_passA", "passB": "spec_passB",
           "carry": "spec_carry", "pin": "spec_pin"}


def per_kernel(path, counter):
    acc = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            for k, sub in KERNELS.items():
                if sub in row["Kernel_Name"]:
                    acc.setdefault(k, []).append(float(row["Counter_Value"]))
    # the first two dispatches of the tendency kernel are the Euler steps (2 words/pt/layer
    # less traffic than AB3): skip them so the mean is over AB3 launches only
    acc = {k: (v[2:] if len(v) > 2 else v) for k, v in acc.items()}
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    tag, n = sys.argv[1], int(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles", "pmc_tendency.json")
    g = os.path.join(ROOT, "gpurun_out")
    fetch, nf = per_kernel(os.path.join(g, f"pmc_{tag}_fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write, nw = per_kernel(os.path.join(g, f"pmc_{tag}_write", "write_counter_collection.csv"), "WRITE_SIZE")
    kern = {}
    for k in KERNELS:
        if k in fetch and k in write:
            rd = 2 * fetch[k] * 1024
            wr = write[k] * 1024
            kern[k] = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
                       "launches_sampled": min(nf[k], nw[k])}
    res = {"n": n, "tag": tag, "source": f"rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                                         f"bench.py --n {n}",
           "correction": "KiB -> bytes; FETCH_SIZE x2 (gfx950 half-count); WRITE_SIZE x1",
           "kernel": "tendency", "hbm_bytes_per_launch": kern.get("tendency", {}).get("hbm_bytes_per_launch"),
           "kernels": kern}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
