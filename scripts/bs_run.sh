set -o pipefail
mkdir -p gpurun_out
L=quic-fec-eps_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "bitslice or encode_decode_vs_oracle or golden or split or ragged or full_size" > gpurun_out/bs_tests.log 2>&1 || { tail -30 gpurun_out/bs_tests.log; exit 1; }
tail -2 gpurun_out/bs_tests.log
V=""; for u in 2 4 8; do for s in 0 1; do V="$V,$L/libfecgpu_u${u}s${s}.so"; done; done; V=${V#,}
{ timeout -k 10 300 python scripts/bs_probe.py --libs $V --codes 16x8,32x8 && timeout -k 10 300 python scripts/bs_probe.py --codes 8x8,24x8; } > gpurun_out/bs_probe4.txt 2>&1 || { cat gpurun_out/bs_probe4.txt; exit 1; }
cat gpurun_out/bs_probe4.txt
A=""; for u in 2 4 8; do for s in 0 1; do A="$A,$L/libfecgpu_u${u}s${s}.so"; done; done; A=${A#,}
timeout -k 10 400 python scripts/ab.py --config 4 --rounds 3 --libs $A > gpurun_out/bs_ab4b.txt 2>&1; rc=$?; cat gpurun_out/bs_ab4b.txt; exit $rc
