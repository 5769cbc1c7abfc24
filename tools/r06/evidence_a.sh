#!/bin/bash
# round-6 evidence, part A (final tree): smoke, the driver's bench command three times on one
# box, the default bench, rocprofv3 kernel stats of the driver's workload, PMC passes.
TAG=${1:-r06e}
R=$GRAFT_REPO_ROOT; cd $R || exit 1
O=gpurun_out/ev_$TAG; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
tail -1 $O/smoke.log
for k in 1 2 3; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$k.json 2> $O/bench_driver_$k.err || exit 3
done
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 3
python - <<PY | tee $O/summary.txt
import json
for f in ["$O/bench_driver_%d.json" % k for k in (1, 2, 3)] + ["$O/bench_default.json"]:
    d = json.loads(open(f).read())
    print(f.split("/")[-1], round(d["value"], 1), "steps/s", round(d["ms_per_step"], 4), "ms/step; tendency",
          round(d["roofline"]["avg_launch_ms"] * 1e3, 1), "us frac", round(d["roofline"]["frac"], 3), "traffic",
          d["roofline"]["traffic"], "; step frac", round(d["step_roofline"]["frac"], 3), "solve",
          round(d["step_roofline"]["solve_ms"] * 1e3, 1), "us; dropin", round(d["dropin"]["vs_qg_run_step"], 3),
          "slot1", round(d["dropin_slot1"]["vs_qg_run_step"], 3), "slot1_deferred",
          round(d["dropin_slot1_deferred"]["vs_qg_run_step"], 3), "; pcg", round(d["pcg_solver"]["value"], 1),
          "; mg-pcg", round(d["mg_pcg_solver"]["value"], 1), d["mg_pcg_solver"]["iters_per_step"][-1],
          "; cpu", round(d["cpu_baseline"]["value"], 3), d["cpu_baseline"]["cores"])
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o drv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc-live --no-reference-runs --cpu-steps 0 --mg-steps 0 > $R/$O/prof.log 2>&1 || exit 4
cut -d, -f1-4 $R/$O/prof/drv_kernel_stats.csv | head -8 | tee -a $R/$O/summary.txt
cd $R && bash tools/pmc.sh ev_$TAG > $O/pmc.log 2>&1 || exit 5
echo done | tee -a $O/summary.txt
