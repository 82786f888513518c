set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1 2; do
for ev in 0 1; do
  a=""; [ $ev = 0 ] && a="--no-kernel-events"
  timeout -k 10 120 python bench.py --config 2 --steps 50 --warmup 5 --cpu-seconds 0 --no-verify $a > gpurun_out/ev_$ev.log 2>&1 || exit $?
  echo "ev=$ev $(grep -o '"ms_per_step": [0-9.]*\|"kernels_ms": {[^}]*}' gpurun_out/ev_$ev.log | tr '\n' ' ')"
done; done
