#!/bin/bash
# Round-4 GPU steps: gpurun --timeout T -- 'bash tools/gpu_r04.sh <step>...'
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
export KRK_DEFAULTS_JSON=gpurun_out/defaults.json
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
for step in "$@"; do
    case $step in
    new) run pytest_new 420 $PYT tests/test_gpu_errors.py tests/test_gpu_defaults.py tests/test_gpu_files.py ;;
    rest) run pytest_rest 600 $PYT tests -m gpu --deselect tests/test_gpu_files.py --deselect tests/test_gpu_defaults.py --deselect tests/test_gpu_errors.py ;;
    all) run pytest_all 900 $PYT tests -m gpu ;;
    crossover) run crc_crossover 300 tests/native/crc_crossover ;;
    defaults) run pytest_defaults 300 $PYT tests/test_gpu_defaults.py tests/test_gpu_bindings.py ;;
    bench) run bench_c2 300 python bench.py ;;
    bench_c1) run bench_c1 300 python bench.py --workload c1 --steps 2 --warmup 1 ;;
    bench_files) run bench_files 600 python bench.py --workload files --steps 2 --warmup 1 ;;
    bench_engine) run bench_engine 300 python bench.py --workload engine ;;
    bench_c4) run bench_c4 600 python bench.py --workload c4 ;;
    bench_c5regen) run bench_c5regen 600 python bench.py --workload c5regen ;;
    bench_f1) run bench_f1verify 600 python bench.py --workload f1verify ;;
    verify_tests) run pytest_verify 400 $PYT tests/test_gpu_agent_verify.py tests/test_gpu_files.py -k "split or placements or verify" ;;
    bench_c3) run bench_c3 900 python bench.py --workload c3 ;;
    bench_c5) run bench_c5 300 python bench.py --workload c5 ;;
    bench_c5regen_digest) run bench_c5regen_digest 400 python bench.py --workload c5regen_digest ;;
    pinned_ab) run pinned_ab 400 python tools/pinned_ab.py 48 192 ;;
    e2e_w2 | e2e_w3 | e2e_w4) run $step 300 env KRK_STAGING_WINDOWS=${step#e2e_w} python bench.py --e2e-only --no-cpu-baseline ;;
    # rocprofv3 on the end-to-end legs (kernel trace + copy trace; PMC passes on their own runs)
    prof_e2e) run prof_e2e 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
                  -d gpurun_out/prof_e2e -- python3 bench.py --e2e-only --no-cpu-baseline ;;
    prof_c2) run prof_c2 400 rocprofv3 --kernel-trace --stats --output-format csv \
                  -d gpurun_out/prof_c2 -- python3 bench.py --no-e2e --no-cpu-baseline ;;
    prof_files) run prof_files 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
                  -d gpurun_out/prof_files -- python3 bench.py --workload files --steps 1 --warmup 1 --no-cpu-baseline ;;
    pmc_c2 | pmc_e2e | pmc_files)
        case $step in
        pmc_c2) B="python3 bench.py --steps 1 --warmup 0 --no-e2e --no-cpu-baseline --no-ceiling" ;;
        pmc_e2e) B="python3 bench.py --e2e-only --no-cpu-baseline" ;;
        pmc_files) B="python3 bench.py --workload files --steps 1 --warmup 0 --no-cpu-baseline" ;;
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
