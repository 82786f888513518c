set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 200 python scripts/sw_bench.py 2>/dev/null | grep '^{' | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['encode_ms'], d['decode_wall_ms'], d['verify_ok'], d['recovered'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/swprof -o run -- python scripts/sw_bench.py > gpurun_out/swprof.log 2>&1
python - <<'P'
import csv
for r in csv.DictReader(open('gpurun_out/swprof/run_kernel_stats.csv')):
    if 'fecgpu' in r['Name']: print(r['Name'][:60], r['Calls'], r['AverageNs'])
P
