set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count(), 'OMP', os.environ.get('OMP_NUM_THREADS'))"
timeout -k 10 600 python -u -m pytest tests/test_gpu_conn_parity.py tests/test_gpu_conn.py tests/test_gpu_boundscheck.py "tests/test_gpu_parity.py::test_full_size_roundtrip" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?; tail -30 gpurun_out/t2.log; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/dist2.log 2>&1
rc=$?; tail -5 gpurun_out/dist2.log; echo "dist2 rc=$rc"
