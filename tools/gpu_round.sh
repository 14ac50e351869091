#!/bin/bash
# One gpurun session: GPU parity tests, then the perf probe; stops at the first
# crash/timeout (exit codes other than 0/1 from a step) or GPU fault in its log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
step() {  # step <name> <timeout> <cmd...>  (env assignments before "step" are exported to it)
  local name=$1 t=$2; shift 2
  echo "=== $name" >&2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -5 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  if grep -qiE "memory fault|illegal memory access|memory access fault|device not stable" "gpurun_out/$name.log"; then
    echo "stopping after $name (GPU fault in log)" >&2; exit 3
  fi
  return 0
}
for s in "$@"; do
  case $s in
    test) step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
    dbg) step dbg_unaligned 300 env KRK_LIB_PATH=kraken_amd/lib/debug/libkraken_hip.so python -m pytest tests/test_gpu_digest_metainfo.py -k "unaligned or lengths" -v -s -p no:cacheprovider ;;
    dbgall) step dbg_digest_all 600 env KRK_LIB_PATH=kraken_amd/lib/debug/libkraken_hip.so python -m pytest tests/test_gpu_digest_metainfo.py -v -s -x -p no:cacheprovider ;;
    serial) step serial_digest 600 env AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 AMD_LOG_LEVEL=1 python -m pytest tests/test_gpu_digest_metainfo.py -v -s -x -p no:cacheprovider ;;
    serial4) step serial_unaligned 300 env KRK_TEST_VERBOSE=1 AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 AMD_LOG_LEVEL=4 python -m pytest tests/test_gpu_digest_metainfo.py -k unaligned -v -s -x -p no:cacheprovider ;;
    hrw) step pytest_hrw 600 python -m pytest tests/test_gpu_hrw.py -x -q -p no:cacheprovider ;;
    pieces) step pytest_pieces 600 python -m pytest tests/test_gpu_pieces.py -x -q -p no:cacheprovider ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    probe0) step probe_v0 300 python tools/probe_perf.py --variant 0 ;;
    probe1) step probe_v1 300 python tools/probe_perf.py --variant 1 --sha none ;;
    shaA) step probe_sha0 300 python tools/probe_perf.py --sha-variant 0 --crc-gb 1 --sha 1024:8,16384:1 ;;
    shaB) step probe_sha1 300 python tools/probe_perf.py --sha-variant 1 --crc-gb 1 --sha 64:8,1024:8,16384:1 ;;
    pmcsha) step pmc_sha_a 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $R/gpurun_out/pmc_sha_a -- python3 $R/tools/probe_perf.py --crc-gb 0 --sha 1024:8 &&
            step pmc_sha_b 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/pmc_sha_b -- python3 $R/tools/probe_perf.py --crc-gb 0 --sha 1024:8 &&
            step pmc_sha_c 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/pmc_sha_c -- python3 $R/tools/probe_perf.py --crc-gb 0 --sha 1024:8 ;;
    micro) step micro_banks 120 tools/micro/vgpr_banks ;;
    micro2) step micro_sha2lane 120 tools/micro/sha2lane ;;
    hwid) step micro_hwid 120 tools/micro/hwid ;;
    vop) step micro_vopcost 120 tools/micro/vopcost ;;
    regrot) step micro_regrot 120 tools/micro/regrot ;;
    cyc) step sha_cycles 300 env KRK_LIB_PATH=kraken_amd/lib/cycles/libkraken_hip.so python tools/probe_perf.py --sha-variant 4 --crc-gb 0 --sha 64:8 &&
         step sha_cycles_real 300 env KRK_LIB_PATH=kraken_amd/lib/cycles/libkraken_hip.so python tools/probe_perf.py --sha-variant 3 --crc-gb 0 --sha 64:8 ;;
    sha2) step probe_sha2 300 python tools/probe_perf.py --sha-variant 3 --crc-gb 0 --sha 64:8,1000:8,4096:4,16384:2 &&
          step probe_sha2t 300 python tools/probe_perf.py --sha-variant 4 --crc-gb 0 --sha 64:8,1000:8 &&
          step probe_sha1b 300 python tools/probe_perf.py --sha-variant 1 --crc-gb 0 --sha 4096:4,16384:2 ;;
    shaP) step probe_shaP 300 python tools/probe_perf.py --sha-variant 6 --crc-gb 0 --sha 64:8,1000:8 &&
          step probe_shaPn 300 python tools/probe_perf.py --sha-variant 7 --crc-gb 0 --sha 64:8,1000:8 &&
          step probe_shaP1 300 python tools/probe_perf.py --sha-variant 5 --crc-gb 0 --sha 64:8,1000:8 ;;
    test1) step pytest_gpu_v1 900 env KRK_SHA_VARIANT=1 python -m pytest tests/test_gpu_digest_metainfo.py -x -q -p no:cacheprovider ;;
    shaD) step probe_sha_diag 300 python tools/probe_perf.py --sha-variant 2 --crc-gb 0 --sha 64:8,1024:8 ;;
    c2split) step probe_c2 300 python tools/probe_perf.py --c2 ;;
    benchsmall) step bench_small 300 python bench.py --workload small --cpu-seconds 3 ;;
    bench) step bench 900 python bench.py ;;
    bc1) step bench_c1 600 python bench.py --workload c1 --steps 1 --warmup 1 ;;
    bc3) step bench_c3 900 python bench.py --workload c3 ;;
    bc4) step bench_c4 600 python bench.py --workload c4 ;;
    bc5) step bench_c5 600 python bench.py --workload c5 ;;
    bc5r) step bench_c5regen 900 python bench.py --workload c5regen ;;
    bc5rd) step bench_c5regen_digest 900 python bench.py --workload c5regen_digest --steps 1 --warmup 1 ;;
    files) step probe_files 600 python tools/probe_files.py ;;
    bf1) step bench_f1verify 600 python bench.py --workload f1verify ;;
    prof) step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-ceiling ;;
    pmcf) step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-ceiling ;;
    pmcf4) step pmc_fetch_c4 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch_c4 -- python3 $R/bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline ;;
    pmcw4) step pmc_write_c4 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write_c4 -- python3 $R/bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline ;;
    prof4) step prof_c4 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4 -- python3 $R/bench.py --workload c4 --no-cpu-baseline ;;
    pmcw) step pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-ceiling ;;
    pmcf5) step pmc_fetch_c5r 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch_c5r -- python3 $R/bench.py --workload c5regen --regen-serial --steps 1 --warmup 0 --no-cpu-baseline ;;
    pmcw5) step pmc_write_c5r 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write_c5r -- python3 $R/bench.py --workload c5regen --regen-serial --steps 1 --warmup 0 --no-cpu-baseline ;;
    prof5) step prof_c5r 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5r -- python3 $R/bench.py --workload c5regen --no-cpu-baseline ;;
    prof5h) step prof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -- python3 $R/bench.py --workload c5 --no-cpu-baseline --no-sweep ;;
    proff1) step prof_f1 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_f1 -- python3 $R/bench.py --workload f1verify --no-cpu-baseline ;;
    prof3) step prof_c3 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3 -- python3 $R/bench.py --workload c3 --no-cpu-baseline ;;
    pmc5) step pmc_fetch_c5 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch_c5 -- python3 $R/bench.py --workload c5 --steps 2 --warmup 0 --no-cpu-baseline --no-sweep &&
          step pmc_write_c5 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write_c5 -- python3 $R/bench.py --workload c5 --steps 2 --warmup 0 --no-cpu-baseline --no-sweep ;;
    pmcpair) for v in 3 4; do
              step pmc_pair_v${v}_a 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/pmc_pair_v${v}_a -- python3 $R/tools/probe_perf.py --sha-variant $v --crc-gb 0 --sha 1000:8 &&
              step pmc_pair_v${v}_b 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY --output-format csv -d $R/gpurun_out/pmc_pair_v${v}_b -- python3 $R/tools/probe_perf.py --sha-variant $v --crc-gb 0 --sha 1000:8 &&
              step pmc_pair_v${v}_c 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC --output-format csv -d $R/gpurun_out/pmc_pair_v${v}_c -- python3 $R/tools/probe_perf.py --sha-variant $v --crc-gb 0 --sha 1000:8 || exit 1; done ;;
  esac
done
