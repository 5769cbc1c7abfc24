# A/B of tendency-kernel variants, F32 states (tendency_pair_kernel) at 4096^2 and 8192^2
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_tendency_kernels.py tests/test_gpu_f32.py > gpurun_out/t_tf.log 2>&1; rc=$?; tail -3 gpurun_out/t_tf.log; [ $rc -ne 0 ] && exit $rc
bash tools/prof_variants.sh f4k --dtype f32 --warmup 20 || exit 3
bash tools/prof_variants.sh f8k --n 8192 --dtype f32 --warmup 5 || exit 4
exit 0
