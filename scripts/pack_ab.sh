# four-column runtime-mask encode index formats: packed dword per plane (default, FECGPU_RBS4_PACK=1), byte per index (2), two dwords per plane (0)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for lib in libfecgpu libfecgpu_pack2 libfecgpu_pack0; do
    FECGPU_LIB=quic-fec-eps_amd/lib/$lib.so timeout -k 10 300 python scripts/code_sweep.py rbs 2>/dev/null | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$lib', d['matrix'], d['k'], d['r'], d['encode_ms'], d['encode_TBps'], d['verify_ok'])"
  done
done
