#!/bin/bash
# C2 end-to-end leg: copy threads sharing the CPU budget with the host offload (default)
# vs 16 copy threads beside it (KRK_COPY_THREADS=16, the round-3 behaviour), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pass in 1 2; do
  for mode in share old; do
    if [ $mode = old ]; then e="KRK_COPY_THREADS=16"; else e=""; fi
    env $e timeout -k 10 300 python bench.py --e2e-only --no-cpu-baseline > gpurun_out/e2e_$mode.log 2>&1 || { echo "rc=$? $mode"; tail -3 gpurun_out/e2e_$mode.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/e2e_$mode.log') if l.startswith('{')][-1]); e=d['end_to_end']; print('$mode', $pass, e['value'], e['passes_s'], e['host_hybrid']['value'], e['host_hybrid']['passes_s'], e['host_hybrid']['outputs_match_gpu_only'])"
  done
done
