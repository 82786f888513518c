# host AddressSanitizer + UBSan over the per-connection objects and frame code
# (library host code built with -Xarch_host -fsanitize=..., kernels unchanged;
# GPU ASan is not available on this pool)
set -o pipefail
mkdir -p gpurun_out
# quarantine off: with it, ROCm's ASan runtime recycles a chunk of its device
# allocator inside the HSA runtime's exit-time finalizer and trips a CHECK
# (dev_runtime_unloaded_) after main() returned
export ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:halt_on_error=1:abort_on_error=0:quarantine_size_mb=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
run() { echo "== $*"; timeout -k 10 180 "$@" > gpurun_out/asan_last.log 2>&1; rc=$?; tail -3 gpurun_out/asan_last.log; cat gpurun_out/asan_last.log >> gpurun_out/asan_all.log; [ $rc -eq 0 ] || { echo "rc=$rc"; grep -A25 "ERROR: AddressSanitizer\|runtime error" gpurun_out/asan_last.log | head -60; exit $rc; }; }
: > gpurun_out/asan_all.log
run ./scripts/conn_bench_asan xor 8 2 1200 48 0.05 64
run ./scripts/conn_bench_asan xor 4 1 1000 16 0.03 16 0 64 0.02
run ./scripts/conn_bench_asan gf256 16 4 1200 48 0.08 128 1 33 0.01
run ./scripts/conn_bench_asan gf256 32 8 9000 64 0.12 16 1
run ./scripts/conn_bench_asan gf256 5 3 333 4 0.2 3 0 7 0.05
run ./scripts/udp_ring_asan xor 8 2 1200 200000 0.03 256
run ./scripts/udp_ring_asan gf256 16 4 1200 100003 0.08 128
echo "asan: all clean"
