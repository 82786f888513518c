# cfg2 XOR: persistent workgroups per CU (bench --bpc), interleaved twice
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for b in 1 2 3 4; do
    timeout -k 10 200 python bench.py --config 2 --steps 200 --warmup 20 --cpu-seconds 0 --no-verify --bpc $b 2>/dev/null | grep '^{' | python -c "import json,sys;d=json.loads(sys.stdin.read());print('bpc', $b, d['value'], d['kernels_ms'])"
  done
done
