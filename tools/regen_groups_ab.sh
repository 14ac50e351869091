#!/bin/bash
# C5 regen (krk_metainfo_batch_dev): CRC groups a call (KRK_REGEN_GROUPS), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pass in 1 2; do
  for g in 8 4 2 1; do
    KRK_REGEN_GROUPS=$g timeout -k 10 200 python bench.py --workload c5regen --no-cpu-baseline > gpurun_out/rg.log 2>&1 || { echo "rc=$? for $g"; tail -3 gpurun_out/rg.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/rg.log') if l.startswith('{')][-1]); print('groups', $g, 'pass', $pass, d['value'], d['ms_per_step'], d['kernels']['crc32_pieces']['avg_ms'], d.get('info_hash_matches_oracle'))"
  done
done
