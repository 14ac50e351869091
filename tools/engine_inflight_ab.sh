#!/bin/bash
# Owner in-flight depth (KRK_OWNER_INFLIGHT) on the 256-digester harness: the burst of
# slot fills at a round's start starves the engine's dispatcher of CPU (tools/engine_slow.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/engine_inflight.jsonl
: > $out
for pass in 1 2; do
  for k in 8 4 3 2; do
    KRK_OWNER_INFLIGHT=$k timeout -k 10 120 tests/native/digesters 256 16 8 > gpurun_out/eif.log 2>&1 || { echo "rc=$? for $k"; tail -3 gpurun_out/eif.log; exit 1; }
    grep '^{' gpurun_out/eif.log | sed "s/^{/{\"owner_inflight\": $k, \"pass\": $pass, /" >> $out
  done
done
python3 - <<'P'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/engine_inflight.jsonl")]
by = collections.defaultdict(list)
for r in rows:
    if r["round"] > 0:
        by[r["owner_inflight"]].append(r["GBps"])
for k, v in sorted(by.items()):
    v = sorted(v)
    print(k, "median %.2f min %.2f max %.2f" % (v[len(v) // 2], v[0], v[-1]), v)
P
