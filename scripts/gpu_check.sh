#!/bin/bash
# One gpurun call: smoke, GPU parity tests, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a fault/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 15 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 3 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
    return 0
}
WHAT=${1:-all}
if [ "$WHAT" = all ] || [ "$WHAT" = test ] || [ "$WHAT" = first ]; then
    step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
    step pytest 1200 python -m pytest tests -m gpu -x -q -p no:cacheprovider
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ] || [ "$WHAT" = first ]; then
    step bench2 600 python bench.py --config 2 --steps 20 --warmup 3
    [ "$WHAT" = first ] || step bench3 600 python bench.py --config 3 --steps 10 --warmup 2 --cpu-seconds 5
    [ "$WHAT" = first ] || step bench4 600 python bench.py --config 4 --steps 5 --warmup 1 --cpu-seconds 5
    step prof2 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof2 -o run -- python bench.py --config 2 --steps 10 --warmup 2 --cpu-seconds 0
fi
echo "== done"
