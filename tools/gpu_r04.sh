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
    crossover) run crc_crossover 200 tests/native/crc_crossover ;;
    bench) run bench_c2 300 python bench.py ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
