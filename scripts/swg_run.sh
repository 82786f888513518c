# Grouped sliding-window encode jobs: parity tests, then sw_bench per group size
# and the per-connection driver (pinned sources read over PCIe).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sw.py tests/test_gpu_swconn.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/swg_tests.log 2>&1
tail -2 gpurun_out/swg_tests.log
for rep in 1 2; do
  for g in 1 2 4; do
    timeout -k 10 200 python scripts/sw_bench.py --sw-group $g 2>/dev/null | grep '^{' >> gpurun_out/swg_bench.jsonl
  done
done
cat gpurun_out/swg_bench.jsonl
for g in 1 4; do
  for b in 64 256; do
    SW_GROUP=$g timeout -k 10 120 ./scripts/sw_conn_bench 1200 32 8 200 0.02 $b | sed "s/^{/{\"sw_group\": $g, /" >> gpurun_out/swg_conn.jsonl
  done
done
cat gpurun_out/swg_conn.jsonl
