# runtime-mask encode: parity (release + checked builds), the code-shape sweep, cfg4 with RLC rows
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundscheck.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bitslice or rlc or checked" 2>&1 | tail -1
timeout -k 10 600 python scripts/code_sweep.py > gpurun_out/code_sweep.jsonl 2>/dev/null
cat gpurun_out/code_sweep.jsonl
timeout -k 10 200 python bench.py --config 4 --matrix rlc --steps 10 --warmup 3 --cpu-seconds 0 2>/dev/null | grep "^{" > gpurun_out/b4rlc.log
python -c "import json;d=json.loads(open('gpurun_out/b4rlc.log').read());print(d['value'], d['kernels_ms'])"
