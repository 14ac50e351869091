#!/bin/bash
# Round-3 GPU session steps (one gpurun call runs several): each step under its own
# time limit, stopping at the first crash / timeout / GPU fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name $(date +%T)" >&2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >&2
  tail -3 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  if grep -qiE "memory fault|illegal memory access|memory access fault|device not stable" "gpurun_out/$name.log"; then
    echo "stopping after $name (GPU fault in log)" >&2; exit 3
  fi
  return 0
}
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS"
P2="GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_LDS"
C2="--steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-ceiling"
for s in "$@"; do
  case $s in
    test) step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 900 python bench.py ;;
    bench20) step bench20 900 python bench.py --steps 20 --warmup 5 ;;
    c3cap) for c in ${CAPS:-16384 13824 12288}; do step bench_c3_cap$c 600 python bench.py --workload c3 --no-cpu-baseline --no-ceiling --live-cap $c || exit 1; done ;;
    lane) step pytest_lane 300 python -u -m pytest tests/test_gpu_windowed.py -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    c3w8lane) step bench_c3_w8_lane 900 python bench.py --workload c3 --no-cpu-baseline --emulate-world 8 --host-lane ;;
    c3lane) step bench_c3_lane 1100 python bench.py --workload c3 --no-cpu-baseline --host-lane ;;
    c3w8) step bench_c3_w8 600 python bench.py --workload c3 --no-cpu-baseline --emulate-world 8 ;;
    c4pipe) step bench_c4 600 python bench.py --workload c4 ;;
    e2ehyb) step e2e_hybrid 900 env KRK_BENCH_HYBRID=${HYB:-4,8,16} python bench.py --e2e-only --no-cpu-baseline ;;
    testoff) step pytest_offload 300 python -u -m pytest tests/test_gpu_digest_metainfo.py -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k offload ;;
    prof) step prof_c2 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c2 -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-ceiling ;;
    valu) step valu_c2_p1 600 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $R/gpurun_out/valu_c2_p1 -- python3 $R/bench.py $C2 &&
          step valu_c2_p2 600 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d $R/gpurun_out/valu_c2_p2 -- python3 $R/bench.py $C2 &&
          step valu_c2_json 120 python tools/pmc_valu.py --dirs gpurun_out/valu_c2_p1 gpurun_out/valu_c2_p2 --mode device_resident --out gpurun_out/valu_c2.json --what "bench.py C2, one step: krk_metainfo_digest_dev over 1000 x 100 MiB in HBM" ;;
    value2e) step valu_e2e_p1 900 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $R/gpurun_out/valu_e2e_p1 -- python3 $R/bench.py --e2e-only --no-cpu-baseline &&
          step valu_e2e_p2 900 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d $R/gpurun_out/valu_e2e_p2 -- python3 $R/bench.py --e2e-only --no-cpu-baseline &&
          step valu_e2e_json 120 python tools/pmc_valu.py --dirs gpurun_out/valu_e2e_p1 gpurun_out/valu_e2e_p2 --mode end_to_end --out gpurun_out/valu_c2.json --what "bench.py C2 end-to-end leg: krk_metainfo_digest_host over 1000 x 100 MiB in pageable host memory (the step before it, one device-resident step, is included in the device_resident block of its own pass)" ;;
  esac
done
for s in "$@"; do
  case $s in
    vop) step micro_vopcost 120 tools/micro/vopcost ;;
    nd) for cfg in "2048 4" "1024 6" "512 8"; do set -- $cfg; step nd_$1_$2 150 env KRK_SLOT_KB=$1 KRK_OWNER_INFLIGHT=$2 tests/native/digesters 256 16 4 || exit 1; done ;;
    traffic) step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -- python3 $R/bench.py $C2 &&
             step pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -- python3 $R/bench.py $C2 &&
             step pmc_traffic_json 120 python tools/pmc_traffic.py --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --out gpurun_out/pmc_traffic.json ;;
    n2) step bench_n2 600 python bench.py --gpus 2 --rehearse --blobs 200 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e ;;
    pmcf) step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -- python3 $R/bench.py $C2 ;;
    pmcw) step pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -- python3 $R/bench.py $C2 ;;
    bc1) step bench_c1 600 python bench.py --workload c1 --steps 1 --warmup 1 ;;
    prof4) step prof_c4 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4 -- python3 $R/bench.py --workload c4 --no-cpu-baseline ;;
    prof5) step prof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -- python3 $R/bench.py --workload c5 --no-cpu-baseline --no-sweep ;;
    prof3) step prof_c3 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3 -- python3 $R/bench.py --workload c3 --no-cpu-baseline ;;
    bc3) step bench_c3 900 python bench.py --workload c3 ;;
    bc4) step bench_c4 600 python bench.py --workload c4 ;;
    bc5) step bench_c5 600 python bench.py --workload c5 ;;
    bc5r) step bench_c5regen 900 python bench.py --workload c5regen ;;
    bc5rd) step bench_c5regen_digest 900 python bench.py --workload c5regen_digest --steps 1 --warmup 1 ;;
    bf1) step bench_f1verify 600 python bench.py --workload f1verify ;;
    crcspec) step crc_spec 600 python tools/probe_perf.py --crc-spec 16:100:4096,16:256:256 --sha none ;;
  esac
done
