#!/bin/bash
# Per-connection path benchmark cases (scripts/conn_bench.cpp); one JSON line each.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
run() { timeout -k 10 120 ./scripts/conn_bench "$@" || exit $?; }
run xor 4 1 1200 10 0.02 256          # config-1 stand-in: 10 MB, XOR k=4 r=1
run xor 8 2 1200 512 0.05 256
run xor 8 2 1200 512 0.05 4096
run gf256 16 4 1200 512 0.05 1024
run gf256 32 8 9000 512 0.10 256 1    # LENPREFIX, lengths 1..9000
timeout -k 10 120 ./scripts/latency_bench xor 8 2 1200 || exit $?
timeout -k 10 120 ./scripts/latency_bench gf256 16 4 1200 || exit $?
