#!/bin/bash
# End-to-end leg (C2, 1000 x 100 MiB from pageable host memory): staging window size and
# copy-thread sweep, KRK_TRACE phase times.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/e2e_sweep.txt; : > $out
for cfg in ${CFGS:-"512 16" "512 8" "512 4" "512 12" "512 16" "512 8" "512 4" "512 12" "512 16" "512 8"}; do
  set -- $cfg
  echo "== window ${1} MiB, copy threads ${2}" >> $out
  KRK_WINDOW_MB=$1 KRK_COPY_THREADS=$2 KRK_TRACE=1 timeout -k 10 180 python -u bench.py --e2e-only --no-cpu-baseline \
      > gpurun_out/e2e_run.log 2>&1 || { tail -20 gpurun_out/e2e_run.log; exit 1; }
  grep "krk_trace metainfo_digest_host" gpurun_out/e2e_run.log | tail -1 >> $out
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/e2e_run.log') if l.startswith('{')][-1]); e=d['end_to_end']; print('value', e['value'], 'seconds', e['seconds'])" >> $out
done
cat $out
