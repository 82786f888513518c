# bit-sliced encode layouts (flat unit space / adjacent column pairs): parity, probe, A/B
set -o pipefail
mkdir -p gpurun_out
L=quic-fec-eps_amd/lib
for v in f1 f1a g0a; do
  FECGPU_LIB=$L/libfecgpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
     --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/par_$v.log 2>&1 || { tail -30 gpurun_out/par_$v.log; exit 1; }
  tail -1 gpurun_out/par_$v.log
done
timeout -k 10 400 python scripts/bs_probe.py --libs $L/libfecgpu_g0.so,$L/libfecgpu_f1.so,$L/libfecgpu_f1a.so,$L/libfecgpu_g0a.so \
   --codes 16x4,8x2,16x8,32x8 > gpurun_out/bs_layout_probe.txt 2>&1 || { cat gpurun_out/bs_layout_probe.txt; exit 1; }
grep '^{' gpurun_out/bs_layout_probe.txt
timeout -k 10 300 python scripts/ab.py --config 3 --rounds 3 --libs $L/libfecgpu.so,$L/libfecgpu_f1.so,$L/libfecgpu_f1a.so > gpurun_out/bs_layout_ab3.txt 2>&1 || { cat gpurun_out/bs_layout_ab3.txt; exit 1; }
grep '^{' gpurun_out/bs_layout_ab3.txt
timeout -k 10 300 python scripts/ab.py --config 4 --rounds 3 --libs $L/libfecgpu.so,$L/libfecgpu_g0a.so > gpurun_out/bs_layout_ab4.txt 2>&1; rc=$?
grep '^{' gpurun_out/bs_layout_ab4.txt; exit $rc
