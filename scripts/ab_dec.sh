#!/bin/bash
# GF decode A/B (round 2): GPU suite on the default build, then cfg3 / cfg4
# in-process A/B of the default build against lib variants.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=quic-fec-eps_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
libs=$L/libfecgpu.so
for v in "$@"; do libs=$libs,$L/libfecgpu_$v.so; done
for c in 3 4; do
  timeout -k 10 300 python scripts/ab.py --config $c --libs $libs --rounds 5 > gpurun_out/ab_dec$c.log 2>&1
  rc=$?; cat gpurun_out/ab_dec$c.log | tail -8; echo "ab$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
