#!/bin/bash
# Two-lane SHA-256 ring 3 vs 4 producer steps (ring4 build, KRK_LIB_PATH): bit-exact tests
# on the ring4 library, then C3 interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R4=$PWD/kraken_amd/lib/ring4/libkraken_hip.so
KRK_LIB_PATH=$R4 timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_gpu_windowed.py tests/test_gpu_c3_production.py tests/test_gpu_digest_metainfo.py -k "plan or windowed or production" \
  > gpurun_out/ring4_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ring4_tests.log
[ $rc -eq 0 ] || exit $rc
for m in ring4 base ring4 base; do
  if [ $m = ring4 ]; then e="KRK_LIB_PATH=$R4"; else e=""; fi
  env $e timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/c3_$m.log 2>&1 || { echo "rc=$? $m"; tail -3 gpurun_out/c3_$m.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/c3_$m.log') if l.startswith('{')][-1]); print('$m', d['value'], d['ms_per_step'], d['kernels']['sha256_multi'], d['spot_check_matches_one_shot'])"
done
