#!/bin/bash
# Caller-runs SHA dispatch (KRK_ENGINE_CALLER_RUNS) on the 256-digester harness, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/engine_caller.jsonl
: > $out
for pass in 1 2; do
  for c in 1 0; do
    KRK_ENGINE_CALLER_RUNS=$c timeout -k 10 120 tests/native/digesters 256 16 8 > gpurun_out/ecr.log 2>&1 || { echo "rc=$? for $c"; tail -3 gpurun_out/ecr.log; exit 1; }
    grep '^{' gpurun_out/ecr.log | sed "s/^{/{\"caller_runs\": $c, \"pass\": $pass, /" >> $out
  done
done
python3 - <<'P'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/engine_caller.jsonl")]
by = collections.defaultdict(list)
for r in rows:
    if r["round"] > 0:
        by[r["caller_runs"]].append(r["GBps"])
for k, v in sorted(by.items()):
    v = sorted(v)
    print(k, "median %.2f min %.2f max %.2f" % (v[len(v) // 2], v[0], v[-1]), v)
P
