"""LDS tile sweep of the tendency kernel (BASELINE config 3: 4096^2 F64, one MI355X).

For each tile W x R (strip width W threads/points, ~R rows per workgroup; qg_set_form(QG_FORM_TENDENCY_TILE)) and
the default geometry, runs tools/tune_tend.py in a fresh process (HIP-event times of 20
qg_evolve_zeta / qg_evolve_psi launches after 5 warm-up steps) and checks that every tile
produced bit-identical zeta (the tiling only changes the traversal).  Writes one JSON list.
usage: python tools/tile_sweep.py OUT.json [N] [tile,tile,...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TILES = ["64x4", "64x8", "128x4", "128x8", "256x2", "256x4",   # SURVEY 8(d) config-3 list
         "64x64", "128x16", "128x64", "256x16", "256x32", "256x64", "256x128", "512x16", "512x64"]


def main():
    out = sys.argv[1]
    n = sys.argv[2] if len(sys.argv) > 2 else "4096"
    tiles = sys.argv[3].split(",") if len(sys.argv) > 3 else TILES
    rows = []
    for tile in [None] + tiles:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "tune_tend.py"), n] + ([tile] if tile else []),
                           capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(r.stderr[-2000:], file=sys.stderr)
            sys.exit(r.returncode)
        rec = json.loads(r.stdout.strip().splitlines()[-1])
        rec["tile"] = tile or "default"
        rows.append(rec)
        print(json.dumps(rec), flush=True)
    ref = rows[0]["zeta_sha1"]
    for rec in rows:
        rec["bitwise_equal_to_default"] = rec["zeta_sha1"] == ref
    with open(out, "w") as f:
        json.dump(rows, f, indent=1)
    bad = [r["tile"] for r in rows if not r["bitwise_equal_to_default"]]
    if bad:
        print("tiles with different results:", bad, file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
