set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundscheck.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bitslice or rlc or checked" > gpurun_out/rbs4_tests.log 2>&1 || { tail -30 gpurun_out/rbs4_tests.log; exit 1; }
tail -1 gpurun_out/rbs4_tests.log
bash scripts/rbs_ab.sh
