#!/bin/bash
# round 5 (f): PMC evidence on this tree -- 4096^2 F64 (bench roofline.traffic) and 8192^2 F32
# (config 5's wide-row solve, verdict r04 item 1) -- plus config 5's kernel stats and 3 bench repeats.
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=gpurun_out/r05f; mkdir -p $O
bash tools/pmc.sh r05f --dropin-steps 0 > $O/pmc4k.log 2>&1 || exit 2
python3 tools/pmc_to_json.py r05f 4096 $O/pmc_tendency_r05f.json > $O/pmc4k.txt 2>&1 || exit 3
cat $O/pmc4k.txt | tail -20
bash tools/pmc.sh r05f8k --n 8192 --dtype f32 --dropin-steps 0 > $O/pmc8k.log 2>&1 || exit 4
python3 tools/pmc_summary.py r05f8k > $O/pmc8k_summary.txt 2>&1 || exit 5
tail -40 $O/pmc8k_summary.txt
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --n 8192 --dtype f32 --steps 20 --warmup 5 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $O/b8k_$rep.json 2> $O/b8k_$rep.err || exit 6
  echo "== 8192 f32 $rep $(grep -o '"value": [0-9.]*' $O/b8k_$rep.json | head -1)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof8k -o k8 -- python3 $R/bench.py --n 8192 --dtype f32 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 --steps 20 --warmup 5 > $R/$O/pb8k.json 2> $R/$O/pb8k.err || exit 7
python3 $R/tools/kstats.py $R/$O/prof8k/k8_kernel_stats.csv
