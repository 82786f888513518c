set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bitslice or rlc" > gpurun_out/rbs_tests.log 2>&1
tail -3 gpurun_out/rbs_tests.log
for m in "--matrix rlc" "--matrix rlc --bitslice 0" "--matrix cauchy" "--matrix vandermonde"; do
  timeout -k 10 200 python bench.py --config 4 --steps 10 --warmup 3 --cpu-seconds 0 $m > gpurun_out/rbs_b4.log 2>&1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/rbs_b4.log') if l.startswith('{')][-1]);print('$m', d['value'], d['kernels_ms'], d['verify']['ok'])"
done
