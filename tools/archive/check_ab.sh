set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh r01bh || exit $?
bash tools/prof_variants.sh c4k --warmup 20 || exit 5
bash tools/prof_variants.sh c1k --n 1024 --warmup 20 --steps 200 || exit 6
