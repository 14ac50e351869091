#!/bin/bash
# First-launch quiet window (KRK_SHA_QUIET_US) on the 256-digester harness, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/engine_quiet.jsonl
: > $out
for pass in 1 2; do
  for q in 3000 10000; do
    KRK_SHA_QUIET_US=$q timeout -k 10 120 tests/native/digesters 256 16 8 > gpurun_out/eq.log 2>&1 || { echo "rc=$? for $q"; tail -3 gpurun_out/eq.log; exit 1; }
    grep '^{' gpurun_out/eq.log | sed "s/^{/{\"quiet_us\": $q, \"pass\": $pass, /" >> $out
  done
done
python3 - <<'P'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/engine_quiet.jsonl")]
by = collections.defaultdict(list)
for r in rows:
    if r["round"] > 0:
        by[r["quiet_us"]].append((r["GBps"], r["sha_launches"]))
for k, v in sorted(by.items()):
    g = sorted(x[0] for x in v)
    print(k, "median %.2f min %.2f max %.2f" % (g[len(g) // 2], g[0], g[-1]), "launches", sorted(x[1] for x in v))
P
