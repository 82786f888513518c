# per-connection path A/B: the tree's library vs scripts/_ab_old/libfecgpu.so
# (conn_bench's RUNPATH yields to LD_LIBRARY_PATH), 3 interleaved rounds
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1 2 3; do
 for v in new old; do
  if [ $v = old ]; then export LD_LIBRARY_PATH=$PWD/scripts/_ab_old; else unset LD_LIBRARY_PATH; fi
  for c in "xor 8 2 1200 512 0.05 256" "gf256 16 4 1200 512 0.05 1024" "gf256 32 8 9000 512 0.10 256 1" "gf256 16 4 1350 512 0.05 256 1"; do
    echo -n "$v $c "; timeout -k 10 120 ./scripts/conn_bench $c | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["send_GBps"], d["recv_GBps"], d["corrupt"], d["unrecovered"] == d["expected_unrecovered"])' || exit 1
  done
 done
done
