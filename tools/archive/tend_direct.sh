# cache-resident tendency vs LDS-ring kernel: bitwise check (zeta hash) and timing by size.
# usage: tools/tend_direct.sh
cd $GRAFT_REPO_ROOT
for n in 256 1024 2048; do
  a=$(QG_TEND_DIRECT=0 timeout -k 10 120 python tools/tune_tend.py $n | tail -1 | python -c "import json,sys; print(json.load(sys.stdin)['zeta_sha1'])") || exit 1
  b=$(QG_TEND_DIRECT=1 timeout -k 10 120 python tools/tune_tend.py $n | tail -1 | python -c "import json,sys; print(json.load(sys.stdin)['zeta_sha1'])") || exit 1
  echo "bitwise $n: $([ "$a" = "$b" ] && echo equal || echo DIFFERENT)"
done
for n in 128 256 512 768 1024 1536 2048; do
  for d in 0 1; do
    QG_TEND_DIRECT=$d timeout -k 10 200 python bench.py --n $n --steps 1000 --cpu-steps 0 --pcg-steps 0 > gpurun_out/td.json 2>gpurun_out/td.err || exit 2
    python -c "import json; d=json.loads(open('gpurun_out/td.json').read().strip().splitlines()[-1]); print($n, 'direct', $d, round(d['value'],1), 'tend us', round(d['roofline']['avg_launch_ms']*1e3,1))"
  done
done
