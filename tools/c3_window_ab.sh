#!/bin/bash
# C3 at N=1 with larger device windows (fewer, longer SHA launches), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in 48 96 120 48 96 120; do
  timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline --window-gib $w > gpurun_out/c3w$w.log 2>&1 || { echo "rc=$? w=$w"; tail -3 gpurun_out/c3w$w.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/c3w$w.log') if l.startswith('{')][-1]); print('window', $w, d['value'], d['ms_per_step'], d['config']['windows'], d['kernels']['sha256_multi']['total_ms'], d['spot_check_matches_one_shot'])"
done
