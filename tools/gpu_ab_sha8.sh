#!/bin/bash
# A/B of experiment builds of the SHA-256 consumers against production on one box:
# interleaved launches of the shapes in $SHAPES (default C2: 1,000 streams x 100 MiB),
# then each experiment's bit-exactness on the SHA launch-plan tests.
# Usage: SHAPES=1000:100,16384:8 tools/gpu_ab_sha8.sh <var name>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/ab_sha8_$(echo "$@" | tr ' ' '_').jsonl
: > $OUT
libs="kraken_amd/lib/libkraken_hip.so"
for v in "$@"; do libs="$libs kraken_amd/lib/var_$v/libkraken_hip.so"; done
for r in 1 2 3; do
  for lib in $libs; do
    timeout -k 10 200 env KRK_LIB_PATH=$lib python tools/probe_perf.py --crc-gb 0 --sha ${SHAPES:-1000:100} > gpurun_out/ab_tmp.log 2>&1 || exit 1
    grep '"sha"' gpurun_out/ab_tmp.log | sed "s|^|{\"lib\": \"$lib\", \"run\": $r, \"r\": |; s|$|}|" >> $OUT
  done
done
for v in "$@"; do
  timeout -k 10 300 env KRK_LIB_PATH=kraken_amd/lib/var_$v/libkraken_hip.so python -m pytest tests/test_gpu_digest_metainfo.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "plans or lengths or stream or offload" > gpurun_out/ab_test_$v.log 2>&1 || { tail -5 gpurun_out/ab_test_$v.log; exit 1; }
  tail -1 gpurun_out/ab_test_$v.log
done
