#!/bin/bash
# One gpurun call = a list of steps, e.g.
#   gpurun -- 'bash scripts/gpu_check.sh smoke pytest bench2 prof2'
# Each GPU step has its own time limit; a fault / abort / timeout stops the
# script (no further GPU work in that call).  Test failures (rc 1) continue.
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
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 3 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
    # a test killed by pytest-timeout may leave its kernel on the card: no more GPU work
    if grep -q "+++ Timeout +++" "gpurun_out/$name.log"; then
        echo "stopping after $name (a test timed out)"
        exit 124
    fi
    return 0
}
prof() {  # name config extra-args...
    local name=$1 cfg=$2; shift 2
    step "$name" 600 rocprofv3 --kernel-trace --stats -f csv -d "gpurun_out/$name" -o run -- \
        python bench.py --config "$cfg" --steps 20 --warmup 10 --cpu-seconds 0 --extra-configs 0 "$@"
}
pmc() {  # name config counters...
    local name=$1 cfg=$2; shift 2
    step "$name" 600 rocprofv3 --kernel-trace --pmc "$@" -f csv -d "gpurun_out/$name" -o run -- \
        python bench.py --config "$cfg" --steps 3 --warmup 1 --cpu-seconds 0 --no-verify --extra-configs 0
}
[ $# -eq 0 ] && set -- smoke pytest bench2 prof2
for s in "$@"; do
    case $s in
        smoke) step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
        pytest) step pytest 1100 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        pytest-x) step pytest 1100 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        bench2) step bench2 600 python bench.py ;;
        bench3) step bench3 600 python bench.py --config 3 --steps 10 --warmup 2 --cpu-seconds 10 ;;
        bench4) step bench4 600 python bench.py --config 4 --steps 5 --warmup 1 --cpu-seconds 10 ;;
        bench7) step bench7 600 python bench.py --config 7 --steps 50 --warmup 5 --cpu-seconds 10 ;;
        bench7l10) step bench7l10 600 python bench.py --config 7 --steps 20 --warmup 5 --cpu-seconds 0 --sw-loss 0.1 ;;
        benchw120) step benchw120 600 python bench.py --k 120 --r 8 --steps 10 --warmup 3 --cpu-seconds 0 ;;
        benchw248) step benchw248 600 python bench.py --k 248 --r 8 --steps 10 --warmup 3 --cpu-seconds 0 ;;
        benchwc) for kk in 120 248; do  # the wide lines with their CPU baselines
                step benchwc$kk 600 python bench.py --k $kk --r 8 --steps 10 --warmup 3 --cpu-seconds 10
            done ;;
        profw120) step profw120 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/profw120 -o run -- \
                      python bench.py --k 120 --r 8 --steps 10 --warmup 3 --cpu-seconds 0 ;;
        profw248) step profw248 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/profw248 -o run -- \
                      python bench.py --k 248 --r 8 --steps 10 --warmup 3 --cpu-seconds 0 ;;
        widetests) step widetests 300 python -u -m pytest tests/test_gpu_wide.py -q -x \
                   --timeout 120 --timeout-method thread -p no:cacheprovider ;;
        abwide)  # k + r > 64: default build vs lib/libfecgpu_wide*.so, k 120 and 248, twice
            for rep in 1 2; do
                for kk in 120 248; do
                    step abwide_base_${kk}_$rep 300 python bench.py --k $kk --r 8 --steps 10 --warmup 3 --cpu-seconds 0
                    for v in quic-fec-eps_amd/lib/libfecgpu_wide*.so; do
                        [ -e "$v" ] || continue
                        n=$(basename $v .so); n=${n#libfecgpu_}
                        FECGPU_LIB=$v step abwide_${n}_${kk}_$rep 300 python bench.py --k $kk --r 8 --steps 10 --warmup 3 --cpu-seconds 0
                    done
                done
            done ;;
        bench5) step bench5 600 python bench.py --config 5 --steps 10 --warmup 2 --cpu-seconds 0 ;;
        bench6) step bench6 600 python bench.py --config 6 --steps 10 --warmup 2 --cpu-seconds 0 ;;
        dist2) step dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                   --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 \
                   --dist-backend gloo ;;  # N>1 rehearsal: 2 ranks share the box's GPU
        prof2) step prof2 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof2 -o run -- \
                   python bench.py ;;  # the driver's default command, as is
        swtests) step swtests 300 python -u -m pytest tests/test_gpu_swconn.py tests/test_gpu_sw.py -q -x \
                     --timeout 120 --timeout-method thread -p no:cacheprovider ;;
        swnew) step swnew 240 python -u -m pytest tests/test_gpu_sw.py -q -x -k \
                   "two_repairs or many_repairs or compaction or async_error or log_overflow or long_path or config7_scale or full_size" \
                   --timeout 60 --timeout-method thread -p no:cacheprovider ;;
        streamtests) step streamtests 300 python -u -m pytest tests/test_gpu_swstream.py -q -x \
                     --timeout 120 --timeout-method thread -p no:cacheprovider ;;
        abstream7)  # cfg7: sliding-window encode modes, interleaved twice
            for rep in 1 2; do
                for m in 0 1 2; do
                    step abstream7_m${m}_$rep 300 python bench.py --config 7 --steps 50 --warmup 5 --cpu-seconds 0 --no-verify --sw-stream $m
                done
            done ;;
        absb7)  # cfg7 streaming encode: LDS budget variants (lib/libfecgpu_sb*.so) and C = 2, interleaved twice
            for rep in 1 2; do
                step absb7_base_$rep 300 python bench.py --config 7 --steps 50 --warmup 5 --cpu-seconds 0 --no-verify
                step absb7_c2_$rep 300 python bench.py --config 7 --steps 50 --warmup 5 --cpu-seconds 0 --no-verify --sw-stream 2
                for v in quic-fec-eps_amd/lib/libfecgpu_sb*.so; do
                    [ -e "$v" ] || continue
                    n=$(basename $v .so); n=${n#libfecgpu_}
                    FECGPU_LIB=$v step absb7_${n}_$rep 300 python bench.py --config 7 --steps 50 --warmup 5 --cpu-seconds 0 --no-verify
                done
            done ;;
        abdec)  # GF decode variants: e = r = 8 sweep rows, cfg3, cfg4 (lib/libfecgpu_*.so), interleaved twice
            libs=quic-fec-eps_amd/lib/libfecgpu.so
            for v in quic-fec-eps_amd/lib/libfecgpu_*.so; do
                [ "$(basename $v)" = libfecgpu_check.so ] || libs=$libs,$v
            done
            step abdec_c3 300 python scripts/ab.py --config 3 --libs $libs
            step abdec_c4 300 python scripts/ab.py --config 4 --libs $libs
            for rep in 1 2; do
                step abdec_sweep_base_$rep 300 python scripts/code_sweep.py r8
                for v in quic-fec-eps_amd/lib/libfecgpu_*.so; do
                    n=$(basename $v .so); n=${n#libfecgpu_}
                    case $n in check|trace) continue ;; esac
                    FECGPU_LIB=$v step abdec_sweep_${n}_$rep 300 python scripts/code_sweep.py r8
                done
            done ;;
        prof5) prof prof5 5 ;;
        prof7) prof prof7 7 ;;
        trace7) FECGPU_LIB=quic-fec-eps_amd/lib/libfecgpu_trace.so step trace7 300 python bench.py --config 7 \
                    --steps 3 --warmup 1 --cpu-seconds 0 --no-verify --extra-configs 0 ;;
        prof7l10) prof prof7l10 7 --sw-loss 0.1 ;;
        ablong)  # cfg7 at 10 % loss: sw_long_min values, twice
            for rep in 1 2; do
                for lm in 65 33 17 9; do
                    step ablong_${lm}_$rep 300 python bench.py --config 7 --steps 20 --warmup 5 --cpu-seconds 0 \
                        --no-verify --sw-loss 0.1 --sw-long-min $lm --extra-configs 0
                done
            done ;;
        prof7v)  # cfg7 rocprofv3 of every lib/libfecgpu_*.so variant (no check build)
            for v in quic-fec-eps_amd/lib/libfecgpu_*.so; do
                n=$(basename $v .so); n=${n#libfecgpu_}
                case $n in check|trace) continue ;; esac
                FECGPU_LIB=$v prof prof7_$n 7
            done ;;
        abvar7)  # cfg7: default build vs every lib/libfecgpu_*.so variant (no check build), interleaved 3 times
            for rep in 1 2 3; do
                step abvar7_base_$rep 300 python bench.py --config 7 --steps 50 --warmup 5 --cpu-seconds 0 --no-verify
                for v in quic-fec-eps_amd/lib/libfecgpu_*.so; do
                    n=$(basename $v .so); n=${n#libfecgpu_}
                    case $n in check|trace) continue ;; esac
                    FECGPU_LIB=$v step abvar7_${n}_$rep 300 python bench.py --config 7 --steps 50 --warmup 5 --cpu-seconds 0 --no-verify
                done
            done ;;
        abvar7l10)  # cfg7 at 10 % loss: default build vs every variant, interleaved twice
            for rep in 1 2; do
                step abvar7l10_base_$rep 300 python bench.py --config 7 --steps 20 --warmup 5 --cpu-seconds 0 --no-verify --sw-loss 0.1
                for v in quic-fec-eps_amd/lib/libfecgpu_*.so; do
                    n=$(basename $v .so); n=${n#libfecgpu_}
                    case $n in check|trace) continue ;; esac
                    FECGPU_LIB=$v step abvar7l10_${n}_$rep 300 python bench.py --config 7 --steps 20 --warmup 5 --cpu-seconds 0 --no-verify --sw-loss 0.1
                done
            done ;;
        abgroup)  # cfg7: sliding-window repairs per combine job, interleaved twice
            for rep in 1 2; do
                for gsz in 2 4 8; do
                    step abgroup_g${gsz}_$rep 300 python bench.py --config 7 --steps 50 --warmup 5 --cpu-seconds 0 --no-verify --sw-group $gsz
                done
            done ;;
        prof3) prof prof3 3 ;;
        prof4) prof prof4 4 ;;
        prof4rlc) prof prof4rlc 4 --matrix rlc ;;
        pmcw*)  # pmcw<K>r / pmcw<K>w: FETCH_SIZE / WRITE_SIZE pass of `bench.py --k K --r 8`
            kk=${s#pmcw}; c=${kk: -1}; kk=${kk%?}
            [ "$c" = r ] && ctr=FETCH_SIZE || ctr=WRITE_SIZE
            step pmcw$kk$c 600 rocprofv3 --kernel-trace --pmc $ctr -f csv -d gpurun_out/pmcw$kk$c -o run -- \
                python bench.py --k $kk --r 8 --steps 3 --warmup 1 --cpu-seconds 0 --no-verify ;;
        pmc2r) pmc pmc2r 2 FETCH_SIZE ;;
        pmc2w) pmc pmc2w 2 WRITE_SIZE ;;
        pmc3r) pmc pmc3r 3 FETCH_SIZE ;;
        pmc3w) pmc pmc3w 3 WRITE_SIZE ;;
        pmc4r) pmc pmc4r 4 FETCH_SIZE ;;
        pmc4w) pmc pmc4w 4 WRITE_SIZE ;;
        pmc7r) pmc pmc7r 7 FETCH_SIZE ;;
        pmc7w) pmc pmc7w 7 WRITE_SIZE ;;
        pmc7sq) pmc pmc7sq 7 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
                    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS ;;
        pmc7ic) step pmc7ic 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVE_CYCLES \
                    -f csv -d gpurun_out/pmc7ic -o run -- python bench.py --config 7 --steps 3 --warmup 1 --cpu-seconds 0 \
                    --no-verify --extra-configs 0 ;;
        pmc7sq2) pmc pmc7sq2 7 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT \
                    SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SMEM ;;
        sqa*) c=${s#sqa}; pmc sqa$c $c SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES ;;
        sqb*) c=${s#sqb}; pmc sqb$c $c SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE ;;
        micro) step micro 600 python scripts/microbench.py ;;
        clk*)  # clkN: effective shader clock (GRBM_GUI_ACTIVE / duration) and UTCL1 translation per dispatch
            c=${s#clk}; pmc clk$c $c GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU \
                TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum ;;
        cfg4probe) step cfg4probe 600 python scripts/cfg4_probe.py ABC ;;
        cfg4order) step cfg4order_ad 600 python scripts/cfg4_probe.py AD && step cfg4order_eb 600 python scripts/cfg4_probe.py EB ;;
        listctr) step listctr 120 rocprofv3 -L ;;
        tracex)  # cfg7 plan trace of every lib/libfecgpu_trace*.so (measurement variants)
            for v in quic-fec-eps_amd/lib/libfecgpu_trace*.so; do
                n=$(basename $v .so); n=${n#libfecgpu_}
                FECGPU_LIB=$v step tracex_$n 300 python bench.py --config 7 --steps 3 --warmup 1 --cpu-seconds 0 \
                    --no-verify --extra-configs 0
            done ;;
        gpufix) step gpufix 300 python -u -m pytest tests/test_gpu_gfdec_many.py tests/test_gpu_wide.py tests/test_gpu_sw.py \
                    tests/test_gpu_boundscheck.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        bsdtests) step bsdtests 300 python -u -m pytest tests/test_gpu_gfdec_many.py tests/test_gpu_wide.py tests/test_gpu_boundscheck.py \
                    tests/test_gpu_parity.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        benchdef) step benchdef 900 python bench.py ;;  # the driver's default command
        probe) step probe 300 ./scripts/stream_probe ;;
        layout) step layout 300 ./scripts/layout_probe ;;
        readp) step readp 300 ./scripts/read_probe ;;
        valu) step valu 300 ./scripts/valu_probe ;;
        sweep*)  # sweepN: blocks-per-CU sweep of config N, default lib + every variant lib
            c=${s#sweep}
            step sweep${c}_base 400 python scripts/sweep.py --config $c
            for v in quic-fec-eps_amd/lib/libfecgpu_*.so; do
                [ -e "$v" ] || continue
                n=$(basename $v .so); n=${n#libfecgpu_}
                FECGPU_LIB=$v step sweep${c}_$n 400 python scripts/sweep.py --config $c
            done ;;
        ab*)  # abN: default build vs every lib/libfecgpu_*.so variant, config N, interleaved twice
            c=${s#ab}
            for rep in 1 2; do
                step ab${c}_base_$rep 300 python bench.py --config $c --steps 20 --warmup 3 --cpu-seconds 0 --no-verify
                for v in quic-fec-eps_amd/lib/libfecgpu_*.so; do
                    [ -e "$v" ] || continue
                    n=$(basename $v .so); n=${n#libfecgpu_}
                    FECGPU_LIB=$v step ab${c}_${n}_$rep 300 python bench.py --config $c --steps 20 --warmup 3 --cpu-seconds 0 --no-verify
                done
                step ab${c}_g2_$rep 300 python bench.py --config $c --steps 20 --warmup 3 --cpu-seconds 0 --no-verify --grid-mult 2
            done ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "== done"
