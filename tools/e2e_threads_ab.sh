#!/bin/bash
# C2 end-to-end leg: copy threads (KRK_COPY_THREADS) against the box's 16-CPU quota, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pass in 1 2; do
  for t in 16 14 12 8; do
    KRK_COPY_THREADS=$t timeout -k 10 300 python bench.py --e2e-only --no-cpu-baseline > gpurun_out/e2e_t$t.log 2>&1 || { echo "rc=$? t=$t"; tail -3 gpurun_out/e2e_t$t.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/e2e_t$t.log') if l.startswith('{')][-1]); e=d['end_to_end']; print('copy_threads', $t, 'pass', $pass, e['value'], e['passes_s'], 'hybrid', e['host_hybrid']['value'], e['host_hybrid']['passes_s'])"
  done
done
