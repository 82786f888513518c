# cfg4 with RLC rows (runtime-mask encode, group mode): 256-unit passes per window group (bs_passes)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for p in 8 16 32; do
    timeout -k 10 200 python bench.py --config 4 --matrix rlc --steps 10 --warmup 3 --cpu-seconds 0 --no-verify --bs-passes $p 2>/dev/null | grep '^{' | python -c "import json,sys;d=json.loads(sys.stdin.read());print('passes', $p, d['value'], d['kernels_ms'])"
  done
done
timeout -k 10 200 python bench.py --config 4 --steps 10 --warmup 3 --cpu-seconds 0 2>/dev/null | grep '^{' | python -c "import json,sys;d=json.loads(sys.stdin.read());print('cauchy', d['value'], d['kernels_ms'], d['verify']['ok'])"
