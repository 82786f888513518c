# bit-sliced vs table GF encode at r <= 4 (variant libs with extra compiled codes)
set -o pipefail
mkdir -p gpurun_out
L=quic-fec-eps_amd/lib
timeout -k 10 300 python scripts/bs_probe.py --libs $L/libfecgpu_bsx.so,$L/libfecgpu_bsx4.so --codes 16x4,8x2,8x4,32x4 > gpurun_out/bs_r4_probe.txt 2>&1 || { cat gpurun_out/bs_r4_probe.txt; exit 1; }
cat gpurun_out/bs_r4_probe.txt
timeout -k 10 400 python scripts/ab.py --config 3 --rounds 3 --libs $L/libfecgpu.so,$L/libfecgpu_bsx.so,$L/libfecgpu_bsx4.so > gpurun_out/bs_r4_ab3.txt 2>&1; rc=$?; cat gpurun_out/bs_r4_ab3.txt; exit $rc
