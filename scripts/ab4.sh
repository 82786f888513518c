# cfg4 A/B of every lib/libfecgpu_*.so variant against the default build (in-process, interleaved)
set -o pipefail
mkdir -p gpurun_out
L=quic-fec-eps_amd/lib
A=$L/libfecgpu.so; for v in $L/libfecgpu_*.so; do A="$A,$v"; done
timeout -k 10 500 python scripts/ab.py --config ${1:-4} --rounds ${2:-3} --libs $A > gpurun_out/ab_${1:-4}.txt 2>&1; rc=$?; cat gpurun_out/ab_${1:-4}.txt; exit $rc
