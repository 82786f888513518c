#!/bin/bash
# Config-5 host pipeline sweep: host_direct bitmask x chunk size (bench.py knobs).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for hd in ${HD:-2 3 6 7}; do for mb in ${MB:-64 128 256 512}; do
  timeout -k 10 120 python bench.py --config ${CFG:-5} --steps 10 --warmup 2 --cpu-seconds 0 --no-verify --host-direct $hd --host-chunk-mb $mb > gpurun_out/s5_${hd}_${mb}.log 2>&1 || exit $?
  echo "hd=$hd mb=$mb $(grep -o '"value": [0-9.]*\|"kernels_ms": {[^}]*}' gpurun_out/s5_${hd}_${mb}.log | tr '\n' ' ')"
done; done
