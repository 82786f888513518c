# A/B: combine kernel zero-skip (default) vs FECGPU_COMB_SKIP=0, sliding-window encode per group size
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sw.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/swg_tests.log 2>&1
tail -1 gpurun_out/swg_tests.log
for rep in 1 2; do
  for lib in libfecgpu libfecgpu_noskip; do
    for g in 1 2 4; do
      FECGPU_LIB=quic-fec-eps_amd/lib/$lib.so timeout -k 10 200 python scripts/sw_bench.py --sw-group $g 2>/dev/null | grep '^{' | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$lib', d['sw_group'], d['encode_ms'], d['decode_wall_ms'], d['verify_ok'])"
    done
  done
done
