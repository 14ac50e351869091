#!/bin/bash
# Round-3 (second session) GPU steps: event-query probe, the windowed / concurrency tests,
# the 256-digester engine trace (zero-copy and H2D slots), host-lane probes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>: stop at a crash / timeout / GPU fault
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
for s in "$@"; do
  case $s in
    evq) step evq 60 tools/micro/evq_probe ;;
    wtest) step wtest 400 python -u -m pytest tests/test_gpu_windowed.py tests/test_gpu_concurrency.py -x -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    test) step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    nd) step nd_zc 120 env KRK_ENGINE_TRACE=1 tests/native/digesters 256 16 3 &&
        step nd_h2d 120 env KRK_SHA_ZERO_COPY=0 tests/native/digesters 256 16 3 ;;
    lane) for p in 0 1 -1; do step lane_p$p 200 env KRK_TRACE=1 KRK_SA_PRIO=$p python tools/lane_probe.py --mode windows --k 480 || exit 1; done ;;
    bench) step bench 900 python bench.py ;;
    prioab) for p in 0 -1 0 -1; do step c2_p$p 300 env KRK_SA_PRIO=$p python bench.py --no-cpu-baseline --no-e2e --no-ceiling || exit 1; done
            for p in 0 -1; do step c3_p$p 300 env KRK_SA_PRIO=$p python bench.py --workload c3 --no-cpu-baseline || exit 1; done ;;
    c3w8lane) step c3w8lane_p-1 600 env KRK_SA_PRIO=-1 python bench.py --workload c3 --no-cpu-baseline --emulate-world 8 --host-lane ;;
    c3lane) step c3lane_p-1 900 env KRK_SA_PRIO=-1 python bench.py --workload c3 --no-cpu-baseline --host-lane ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  esac
done
