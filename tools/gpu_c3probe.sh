#!/bin/bash
# SHA plans at C3-like stream counts, alone and beside the CRC kernel (probe_perf.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/c3probe.jsonl
: > $O
for p in ${PLANS-2 4 3 1 5 6}; do
  timeout -k 10 240 python tools/probe_perf.py --sha-plan $p --crc-gb 0 --sha ${SHA-4096:8,8192:4,16384:2,32768:1} >> $O 2> gpurun_out/c3probe_$p.err || exit $?
  echo "plan $p done" >&2
done
for p in ${SPLITPLANS-4 5}; do
  timeout -k 10 240 python tools/probe_perf.py --sha-plan $p --split ${SPLIT-16384:2:1024,4096:8:4096} >> $O 2>> gpurun_out/c3probe_$p.err || exit $?
done
cat $O
