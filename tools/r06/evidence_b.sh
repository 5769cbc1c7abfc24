#!/bin/bash
# round-6 evidence, part B (final tree): BASELINE config 5 (8192^2 F32) three times on one box
# with its rocprofv3 kernel stats; the multi-GPU bench path on the one GPU (2 ranks over RCCL
# loopback, probe group first) at config 3/4's and config 5's per-GPU sizes; the 1-rank RCCL
# ring (--comm-self) against the plain path.
TAG=${1:-r06f}
R=$GRAFT_REPO_ROOT; cd $R || exit 1
O=gpurun_out/ev_$TAG; mkdir -p $O
B="--cpu-steps 0 --cpu-steps-1t 0 --pcg-steps 0 --mg-steps 0 --dropin-steps 0 --no-pmc-live --no-reference-runs"
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --n 8192 --dtype f32 --steps 50 --warmup 5 $B > $O/c5_$k.json 2> $O/c5_$k.err || exit 1
done
timeout -k 10 400 python bench.py --gpus 2 --one-gpu --steps 20 --warmup 5 $B > $O/two_rank_4096.json 2> $O/two_rank_4096.err || exit 2
timeout -k 10 400 python bench.py --gpus 2 --one-gpu --n 8192 --dtype f32 --steps 20 --warmup 5 $B > $O/two_rank_8192f32.json 2> $O/two_rank_8192f32.err || exit 3
timeout -k 10 300 python bench.py --comm-self --steps 50 --warmup 5 $B > $O/commself.json 2> $O/commself.err || exit 4
timeout -k 10 300 python bench.py --steps 50 --warmup 5 $B > $O/plain.json 2> $O/plain.err || exit 4
python - <<PY | tee $O/summary.txt
import json
def rd(f):
    return json.loads(open("$O/" + f).read())
for k in (1, 2, 3):
    d = rd(f"c5_{k}.json"); r = d["step_roofline"]
    print(f"config 5 run {k}: {d['value']:.1f} steps/s, {d['ms_per_step']:.4f} ms/step, tendency {r['tendency_ms']*1e3:.1f} us, solve {r['solve_ms']*1e3:.1f} us")
for f in ("two_rank_4096.json", "two_rank_8192f32.json"):
    d = rd(f); c = d["config"]
    print(f"{f}: {d['value']:.1f} steps/s aggregate (2 ranks sharing one GPU: not scaling), probe: {c['transport_probe']}; "
          f"halo {c['halo_transport']} gather {c['gather_transport']}; check: {c['transport_check']}; "
          f"transport_ab {d.get('transport_ab', {}).get('value')}")
a, b = rd("commself.json"), rd("plain.json")
print(f"1-rank RCCL ring {a['value']:.1f} vs plain {b['value']:.1f} steps/s = {a['value'] / b['value']:.3f}")
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof8k -o c5 -- python3 $R/bench.py --n 8192 --dtype f32 --steps 20 --warmup 5 $B > $R/$O/prof8k.log 2>&1 || exit 5
python3 $R/tools/kstats.py $R/$O/prof8k/c5_kernel_stats.csv | tee -a $R/$O/summary.txt
