# bench.py --config 7 (sliding-window RLC) with its CPU baseline, its GPU test, and a rocprof summary
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_sw.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bench_config7" 2>&1 | tail -1
timeout -k 10 300 python bench.py --config 7 --steps 50 --warmup 5 > gpurun_out/bench7.log 2>gpurun_out/bench7.err
cat gpurun_out/bench7.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof7 -o run -- python bench.py --config 7 --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/prof7.log 2>&1
python - <<'P'
import csv
for r in csv.DictReader(open('gpurun_out/prof7/run_kernel_stats.csv')):
    if 'fecgpu' in r['Name']: print(r['Name'][:60], r['Calls'], r['AverageNs'])
P
