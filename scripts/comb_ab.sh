# grouped sliding-window encode: rows per load batch of the combine kernel (FECGPU_COMB_U_GRP 8 default, 16, 4)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for lib in libfecgpu libfecgpu_cu16 libfecgpu_cu4; do
    FECGPU_LIB=quic-fec-eps_amd/lib/$lib.so timeout -k 10 200 python scripts/sw_bench.py 2>/dev/null | grep '^{' | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$lib', d['encode_ms'], d['decode_wall_ms'], d['verify_ok'])"
  done
done
