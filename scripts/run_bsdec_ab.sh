#!/bin/bash
# Round 6: parity of the bit-sliced syndrome decode, then cfg3 in-process A/B
# against the table decode (the "bsdec" knob).  Tuning aid.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=quic-fec-eps_amd/lib/libfecgpu.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_bsdec.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/bsdec_test.log 2>&1
rc=$?; tail -15 gpurun_out/bsdec_test.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ab.py --config 3 --rounds 5 --libs $L@bsdec=0,$L@bsdec=1,$L@bsdec=0,$L@bsdec=1 > gpurun_out/ab_bsdec.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_bsdec.log; echo "ab rc=$rc"
