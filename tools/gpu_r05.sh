#!/bin/bash
# Round-5 GPU steps: gpurun --timeout T -- 'bash tools/gpu_r05.sh <step>...'
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
for step in "$@"; do
    case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    all) run pytest_all 1000 $PYT tests -m gpu ;;
    new) run pytest_new 600 $PYT tests/test_gpu_files.py tests/test_gpu_digest_metainfo.py tests/test_gpu_bench_contract.py tests/test_gpu_defaults.py tests/test_gpu_bindings.py tests/test_gpu_engine.py ;;
    gather) run gather_probe 240 tools/micro/gather_probe 8 16 ;;
    disk) run disk_info 60 bash -c 'df -h . /tmp /dev/shm; lsblk -o NAME,SIZE,ROTA,TYPE,MOUNTPOINT 2>/dev/null | head -30; free -g; nproc; cat /sys/fs/cgroup/cpu.max; cat /sys/fs/cgroup/memory.max; mount | grep -E " / | /tmp " ; echo; ls -la /mnt /scratch /local 2>/dev/null | head' ;;
    ddtest) run dd_test 300 bash -c 'd=$(mktemp -d -p .); dd if=/dev/zero of=$d/f bs=64M count=96 oflag=direct conv=fsync 2>&1 | tail -1; sync; dd if=$d/f of=/dev/null bs=64M iflag=direct 2>&1 | tail -1; rm -rf $d' ;;
    bench) run bench_c2 300 python bench.py ;;
    bench_engine) run bench_engine 900 python bench.py --workload engine ;;
    bench_engine_zc) run bench_engine_zc 900 env KRK_ENGINE_SLOT_SRC=zerocopy python bench.py --workload engine ;;
    bench_engine_gather) run bench_engine_gather 900 env KRK_ENGINE_SLOT_SRC=gather python bench.py --workload engine ;;
    diskprobe) run disk_probe 400 bash -c 'd=$(mktemp -d -p .); tools/micro/disk_probe $d 32; rc=$?; rm -rf $d; exit $rc' ;;
    hostmem) run host_mem_probe 400 tools/micro/host_mem_probe 8 16 ;;
    regprobe) run reg_probe 300 tools/micro/reg_probe 8 ;;
    gather_tests) run pytest_gather 600 $PYT tests/test_gpu_gather.py tests/test_gpu_files.py tests/test_gpu_agent_verify.py tests/test_gpu_bindings.py tests/test_gpu_bench_contract.py ;;
    engine_tests) run pytest_engine 600 $PYT tests/test_gpu_engine.py tests/test_gpu_concurrency.py tests/test_gpu_bindings.py tests/test_gpu_digest_metainfo.py ;;
    tail_trace) run tail_trace 400 env KRK_TRACE=1 python bench.py --no-e2e --no-cpu-baseline ;;
    hyb_sweep) run hyb_sweep 600 env KRK_BENCH_HYBRID=-1,6,8,10,12 python bench.py --e2e-only --no-cpu-baseline ;;
    bench_defaults) run bench_defaults 300 python bench.py --workload defaults ;;
    bench_files) run bench_files 900 python bench.py --workload files --steps 2 --warmup 1 ;;
    bench_c4) run bench_c4 600 python bench.py --workload c4 ;;
    bench_c3) run bench_c3 900 python bench.py --workload c3 ;;
    bench_c5) run bench_c5 300 python bench.py --workload c5 ;;
    bench_c5regen) run bench_c5regen 600 python bench.py --workload c5regen ;;
    bench_c5regen_digest) run bench_c5regen_digest 400 python bench.py --workload c5regen_digest ;;
    bench_f1) run bench_f1verify 600 python bench.py --workload f1verify ;;
    bench_c1) run bench_c1 300 python bench.py --workload c1 --steps 2 --warmup 1 ;;
    # the LDS-DMA CRC variants live in the diagnostic build (make -C kraken_amd/csrc diag)
    crc_parity) run crc_parity 600 env KRK_CRC_VARIANT=20 KRK_LIB_PATH=kraken_amd/lib/diag/libkraken_hip.so $PYT tests/test_gpu_pieces.py tests/test_gpu_full_size.py tests/test_gpu_digest_metainfo.py ;;
    crc_ab) for v in 16 20 21 16 20 21; do run crc_c4_v$v.$RANDOM 300 env KRK_CRC_VARIANT=$v KRK_LIB_PATH=kraken_amd/lib/diag/libkraken_hip.so python bench.py --workload c4 --no-cpu-baseline --no-e2e; done ;;
    crc_ab2) for v in 16 22 23 16 22 23; do run crc_c4_v$v.$RANDOM 300 env KRK_CRC_VARIANT=$v KRK_LIB_PATH=kraken_amd/lib/diag/libkraken_hip.so python bench.py --workload c4 --no-cpu-baseline --no-e2e; done ;;
    crc_parity22 | crc_parity23) v=${step#crc_parity}
        run crc_parity$v 600 env KRK_CRC_VARIANT=$v KRK_LIB_PATH=kraken_amd/lib/diag/libkraken_hip.so $PYT tests/test_gpu_pieces.py tests/test_gpu_full_size.py ;;
    # rocprofv3 summaries (kernel trace + copy trace; PMC passes on their own runs)
    prof_c5) run prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv \
                  -d gpurun_out/prof_c5 -- python3 bench.py --workload c5 --no-cpu-baseline --no-sweep ;;
    prof_c2) run prof_c2 400 rocprofv3 --kernel-trace --stats --output-format csv \
                  -d gpurun_out/prof_c2 -- python3 bench.py --no-e2e --no-cpu-baseline ;;
    prof_files) run prof_files 600 rocprofv3 --kernel-trace --stats --output-format csv \
                  -d gpurun_out/prof_files -- python3 bench.py --workload files --steps 1 --warmup 1 --cold-gib 0 --no-cpu-baseline ;;
    prof_tail) run prof_tail 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
                  -d gpurun_out/prof_tail -- python3 bench.py --no-e2e --no-cpu-baseline ;;
    prof_e2e) run prof_e2e 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
                  -d gpurun_out/prof_e2e -- python3 bench.py --e2e-only --no-cpu-baseline ;;
    prof_c4) for v in 16 20 21; do run prof_c4_v$v 300 env KRK_CRC_VARIANT=$v KRK_LIB_PATH=kraken_amd/lib/diag/libkraken_hip.so rocprofv3 --kernel-trace --stats --output-format csv \
                  -d gpurun_out/prof_c4_v$v -- python3 bench.py --workload c4 --no-cpu-baseline --no-e2e; done ;;
    # round-5 PMC of the production kernels on the current tree (tools/pmc_traffic.py, pmc_valu.py)
    pmc_c2 | pmc_c4 | pmc_c5 | pmc_files | pmc_e2e)
        case $step in
        pmc_c5) B="python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-sweep" ;;
        pmc_e2e) B="python3 bench.py --e2e-only --no-cpu-baseline" ;;
        pmc_c2) B="python3 bench.py --steps 1 --warmup 0 --no-e2e --no-cpu-baseline --no-ceiling" ;;
        pmc_c4) B="python3 bench.py --workload c4 --steps 3 --warmup 1 --no-e2e --no-cpu-baseline" ;;
        pmc_files) B="python3 bench.py --workload files --steps 1 --warmup 0 --cold-gib 0 --no-cpu-baseline" ;;
        esac
        X=${step#pmc_}
        run pmc_${X}_valu 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
            SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_${X}_valu -- $B
        run pmc_${X}_wait 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc_${X}_wait -- $B
        run pmc_${X}_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${X}_fetch -- $B
        run pmc_${X}_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${X}_write -- $B ;;
    pmc_c4_v16 | pmc_c4_v20 | pmc_c4_v21 | pmc_c4_v22 | pmc_c4_v23)
        v=${step#pmc_c4_v}
        B="python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e"
        run ${step}_valu 300 env KRK_CRC_VARIANT=$v KRK_LIB_PATH=kraken_amd/lib/diag/libkraken_hip.so rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
            SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/${step}_valu -- $B
        run ${step}_wait 300 env KRK_CRC_VARIANT=$v KRK_LIB_PATH=kraken_amd/lib/diag/libkraken_hip.so rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/${step}_wait -- $B ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
