#!/bin/bash
# round 5 (n): the driver's own commands on the committed tree (smoke, bench with its flags).
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 5; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -10 $O/bench_driver.err; exit 6; }
tail -1 $O/bench_driver.json | cut -c1-400
timeout -k 10 400 python tools/r05/f32_scaling.py > $O/f32_scaling.txt 2>&1 || { tail -5 $O/f32_scaling.txt; exit 7; }
cat $O/f32_scaling.txt
