# 8192^2 (BASELINE config 5: F32; and F64) kernel stats with the bench's own steps.
# usage: tools/prof_8k.sh TAG
TAG=${1:-8k}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for dt in f32 f64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_$dt -o ${TAG}_$dt -- python3 $R/bench.py --n 8192 --dtype $dt --steps 30 --warmup 10 --cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --dropin-steps 0 > $R/gpurun_out/prof_${TAG}_$dt.log 2>&1 || exit 5
  cut -d, -f1-4 $R/gpurun_out/prof_${TAG}_$dt/${TAG}_${dt}_kernel_stats.csv | head -8
done
