cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_fuse.log 2>&1; rc=$?; tail -3 gpurun_out/tests_fuse.log; [ $rc -ne 0 ] && exit $rc
bash tools/sweep.sh
