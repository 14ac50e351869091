#!/bin/bash
# Round-6 GPU steps: gpurun --timeout T -- 'bash tools/gpu_r06.sh <step>...'
# Each step runs under its own time limit; a step that ends in a fault, abort, crash or
# time limit (rc >= 2 other than pytest's 1 = test failures) ends the script: nothing more
# runs on the GPU in that call.
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -3 "gpurun_out/$name.log"
    if [ $rc -ge 2 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
C3T="python -u bench.py --workload c3 --emulate-world 8 --c3-tail-only --no-e2e --no-cpu-baseline"
for step in "$@"; do
    case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    all) run pytest_all 1100 $PYT tests -m gpu ;;
    windowed) run pytest_windowed 400 $PYT tests/test_gpu_windowed.py ;;
    bench) run bench_c2 300 python bench.py ;;
    c3w8) run bench_c3_w8 600 python -u bench.py --workload c3 --emulate-world 8 --tail-handoff --host-lane --no-e2e ;;
    c3w8_tail) run bench_c3_w8_tail 200 $C3T ;;
    c3w4) run bench_c3_w4 400 python -u bench.py --workload c3 --emulate-world 4 --tail-handoff --no-e2e --no-cpu-baseline ;;
    c3w2) run bench_c3_w2 400 python -u bench.py --workload c3 --emulate-world 2 --tail-handoff --no-e2e --no-cpu-baseline ;;
    c3) run bench_c3 900 python -u bench.py --workload c3 --tail-handoff ;;
    tail_sweep) for cfg in ${TAIL_SWEEP:-6x64 12x64 16x32}; do set -- ${cfg/x/ }
                    run c3_tail_r$1_p$2 200 $C3T --tail-ring $1 --tail-piece-mib $2; done ;;
    tail_probe) run tail_probe 200 python -u tools/tail_probe.py 15 ;;
    prof_c3w8) run prof_c3w8 400 rocprofv3 --kernel-trace --stats --output-format csv \
                  -d gpurun_out/prof_c3w8 -- python3 bench.py --workload c3 --emulate-world 8 --tail-handoff --no-e2e --no-cpu-baseline --no-ceiling ;;
    prof_c3) run prof_c3 400 rocprofv3 --kernel-trace --stats --output-format csv \
                  -d gpurun_out/prof_c3 -- python3 bench.py --workload c3 --no-e2e --no-cpu-baseline --no-ceiling ;;
    # PMC passes of C3's windows (N=1), each pass its own run (counter limits per block)
    pmc_c3_valu) run pmc_c3_valu 400 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES \
                  SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv \
                  -d gpurun_out/pmc_c3_valu -- python3 bench.py --workload c3 --no-e2e --no-cpu-baseline --no-ceiling ;;
    pmc_c3_wait) run pmc_c3_wait 400 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY \
                  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv \
                  -d gpurun_out/pmc_c3_wait -- python3 bench.py --workload c3 --no-e2e --no-cpu-baseline --no-ceiling ;;
    pmc_c3_hbm) run pmc_c3_hbm 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv \
                  -d gpurun_out/pmc_c3_hbm -- python3 bench.py --workload c3 --no-e2e --no-cpu-baseline --no-ceiling ;;
    # the two-lane plan alone: 14,336 streams of 16 MiB in one device-resident launch (C3's
    # live count), plain and under the PMC pass the C3 windows got
    small2l) run bench_small2l 300 python -u bench.py --workload small --blobs 14336 --no-e2e --no-cpu-baseline --no-offload ;;
    pmc_small2l) run pmc_small2l 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES \
                  SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv \
                  -d gpurun_out/pmc_small2l -- python3 bench.py --workload small --blobs 14336 --no-e2e --no-cpu-baseline --no-ceiling --no-offload --steps 1 --warmup 1 ;;
    pmc_small2l_wait) run pmc_small2l_wait 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY \
                  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv \
                  -d gpurun_out/pmc_small2l_wait -- python3 bench.py --workload small --blobs 14336 --no-e2e --no-cpu-baseline --no-ceiling --no-offload --steps 1 --warmup 1 ;;
    bench_f1) run bench_f1verify 600 python -u bench.py --workload f1verify ;;
    bench_c4) run bench_c4 600 python -u bench.py --workload c4 ;;
    bench_files) run bench_files 900 python -u bench.py --workload files --steps 2 --warmup 1 ;;
    bench_c5) run bench_c5 300 python -u bench.py --workload c5 ;;
    bench_c5regen) run bench_c5regen 600 python -u bench.py --workload c5regen ;;
    bench_c1) run bench_c1 300 python -u bench.py --workload c1 --steps 2 --warmup 1 ;;
    bench_defaults) run bench_defaults 300 python -u bench.py --workload defaults ;;
    prof_c2) run prof_c2 400 rocprofv3 --kernel-trace --stats --output-format csv \
                  -d gpurun_out/prof_c2 -- python3 bench.py --no-e2e --no-cpu-baseline --no-offload ;;
    # final-tree PMC of the production kernels (tools/pmc_traffic.py, pmc_valu.py), each pass its own run
    pmc_c2 | pmc_c4 | pmc_e2e)
        case $step in
        pmc_e2e) B="python3 bench.py --e2e-only --no-cpu-baseline" ;;
        pmc_c2) B="python3 bench.py --steps 1 --warmup 0 --no-e2e --no-cpu-baseline --no-ceiling --no-offload" ;;
        pmc_c4) B="python3 bench.py --workload c4 --steps 3 --warmup 1 --no-e2e --no-cpu-baseline" ;;
        esac
        X=${step#pmc_}
        run pmc_${X}_valu 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
            SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_${X}_valu -- $B
        run pmc_${X}_wait 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_${X}_wait -- $B
        run pmc_${X}_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${X}_fetch -- $B
        run pmc_${X}_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${X}_write -- $B ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
