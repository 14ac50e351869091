#!/bin/bash
# C5 regen: the last CRC group's share of the bytes (KRK_REGEN_TAIL; 0 = equal groups), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pass in 1 2; do
  for t in ${TAILS:-0 0.1 0.04}; do
    KRK_REGEN_TAIL=$t timeout -k 10 200 python bench.py --workload c5regen --no-cpu-baseline > gpurun_out/rt.log 2>&1 || { echo "rc=$? for $t"; tail -3 gpurun_out/rt.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/rt.log') if l.startswith('{')][-1]); print('tail', '$t', 'pass', $pass, d['value'], d['ms_per_step'], d['kernels']['crc32_pieces']['avg_ms'], d.get('info_hash_matches_oracle'))"
  done
done
