#!/bin/bash
# Does the NUMA node of the engine's pinned staging slots (read in place by the SHA-256
# kernel over PCIe) explain the bimodal 256-digester rate?  KRK_SLOT_NUMA unset / 0 / 1,
# interleaved, 8 rounds each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/engine_numa.jsonl
: > $out
for f in /sys/bus/pci/devices/*/numa_node; do :; done
for pass in 1 2; do
  for nm in none 0 1; do
    if [ $nm = none ]; then e=""; else e="KRK_SLOT_NUMA=$nm"; fi
    env $e timeout -k 10 120 tests/native/digesters 256 16 8 > gpurun_out/enuma.log 2>&1 || { echo "rc=$? for $nm"; tail -3 gpurun_out/enuma.log; exit 1; }
    grep '^{' gpurun_out/enuma.log | sed "s/^{/{\"numa\": \"$nm\", \"pass\": $pass, /" >> $out
  done
done
python3 - <<'P'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/engine_numa.jsonl")]
by = collections.defaultdict(list)
for r in rows:
    if r["round"] > 0:
        by[r["numa"]].append(r["GBps"])
for k, v in by.items():
    v = sorted(v)
    print(k, "median %.2f min %.2f max %.2f" % (v[len(v) // 2], v[0], v[-1]), v)
P
