#!/bin/bash
# C3 with the window generator and the SHA-256 launches on disjoint CUs (--cu-split), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in split base split base; do
  if [ $m = split ]; then f=--cu-split; else f=; fi
  timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline $f > gpurun_out/c3_$m.log 2>&1 || { echo "rc=$? $m"; tail -3 gpurun_out/c3_$m.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/c3_$m.log') if l.startswith('{')][-1]); print('$m', d['value'], d['ms_per_step'], d['kernels'], d['spot_check_matches_one_shot'])"
done
