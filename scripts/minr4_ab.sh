# cfg3 (k16 r4): table multiply (default) vs runtime-mask bit-slicing at r = 4 (FECGPU_RBS_MIN_R=4)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for lib in libfecgpu libfecgpu_minr4; do
    for m in cauchy rlc; do
      FECGPU_LIB=quic-fec-eps_amd/lib/$lib.so timeout -k 10 200 python bench.py --config 3 --matrix $m --steps 20 --warmup 3 --cpu-seconds 0 2>/dev/null | grep '^{' | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$lib', '$m', d['value'], d['kernels_ms'], d['verify']['ok'])"
    done
  done
done
