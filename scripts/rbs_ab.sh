# A/B of the runtime bit-sliced encode variants: cfg4 (group mode, per-window S)
# and cfg3-shaped uniform windows with --matrix rlc; interleaved twice.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  FECGPU_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-verify "$@" > gpurun_out/ab_$n.log 2>&1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/ab_$n.log') if l.startswith('{')][-1]);print('$n', '$*', d['value'], d['kernels_ms'])"
}
for rep in 1 2; do
  run base quic-fec-eps_amd/lib/libfecgpu.so --config 4 --matrix rlc
  run table quic-fec-eps_amd/lib/libfecgpu.so --config 4 --matrix rlc --bitslice 0
  for v in pack0; do run $v quic-fec-eps_amd/lib/libfecgpu_$v.so --config 4 --matrix rlc; done
done
run cauchy quic-fec-eps_amd/lib/libfecgpu.so --config 4
