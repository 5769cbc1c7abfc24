#!/bin/bash
# End-of-round evidence, part A: the driver's own commands on this tree (GPU tests, smoke, the
# bench with the driver's flags and with the defaults), rocprof kernel stats of the bench and
# the PMC traffic passes behind roofline.traffic.  usage: tools/round_evidence.sh TAG
TAG=${1:-rc}
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
git_sha=$(cat .gpurun_sha 2>/dev/null || echo unknown)
echo "tree sha: $git_sha" > gpurun_out/evidence_$TAG.txt
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.log | tee -a gpurun_out/evidence_$TAG.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 2
tail -1 gpurun_out/smoke_$TAG.log | tee -a gpurun_out/evidence_$TAG.txt
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_drv.json 2> gpurun_out/bench_${TAG}_drv.err || exit 3
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 3
python - <<PY | tee -a gpurun_out/evidence_$TAG.txt
import json
for f in ("gpurun_out/bench_${TAG}_drv.json", "gpurun_out/bench_${TAG}.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"], 1), "steps/s", round(d["ms_per_step"], 4), "ms", "tend frac", round(d["roofline"]["frac"], 3),
          "step frac", round(d["step_roofline"]["frac"], 3), "dropin", d.get("dropin", {}).get("vs_qg_run_step"))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o $TAG -- python3 $R/bench.py --steps 50 --warmup 20 --cpu-steps 0 --pcg-steps 0 --dropin-steps 0 > $R/gpurun_out/prof_$TAG.log 2>&1 || exit 4
cut -d, -f1-4 $R/gpurun_out/prof_$TAG/${TAG}_kernel_stats.csv | head -6 | tee -a $R/gpurun_out/evidence_$TAG.txt
cd $R && bash tools/pmc.sh $TAG --dropin-steps 0 > gpurun_out/pmc_$TAG.log 2>&1 || exit 5
echo done | tee -a gpurun_out/evidence_$TAG.txt
