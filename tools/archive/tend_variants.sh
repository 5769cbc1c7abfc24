# tendency variants by QG_TEND_VARIANT at 4096^2 (A/B on one box).  usage: tools/tend_variants.sh V...
cd $GRAFT_REPO_ROOT
for v in 0 "$@"; do
  QG_TEND_VARIANT=$v timeout -k 10 200 python bench.py --steps 100 --cpu-steps 0 --pcg-steps 0 > gpurun_out/tv.json 2>gpurun_out/tv.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/tv.json').read().strip().splitlines()[-1]); print('variant', '$v', round(d['value'],1), 'tend us', round(d['roofline']['avg_launch_ms']*1e3,1))"
done
