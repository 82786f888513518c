set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_boundscheck.py -k "wide" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/wide_test.log 2>&1
rc=$?; tail -n 3 gpurun_out/wide_test.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for m in 1 0; do
    for kk in 120 248; do
      timeout -k 10 300 python bench.py --k $kk --r 8 --steps 10 --warmup 3 --cpu-seconds 0 --tune wide_mask=$m > gpurun_out/wide_${kk}_m${m}_$rep.log 2>&1 || exit $?
      python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], d['value'], d['kernels_ms'], d['verify']['ok'] if d.get('verify') else None)" gpurun_out/wide_${kk}_m${m}_$rep.log k${kk}_mask${m}_$rep
    done
  done
done
