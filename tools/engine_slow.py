"""Slow submission steps (krk_engine slow ...) per harness round, beside the round's rate.
    python tools/engine_slow.py gpurun_out/nd_slow.log"""
import collections
import json
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
rounds = [json.loads(l) for l in lines if l.startswith("{")]
slow = [(m.group(1), float(m.group(2)), float(m.group(3))) for l in lines
        for m in [re.match(r"krk_engine slow (\S+) ([\d.]+)ms abs=([\d.]+)ms", l)] if m]
launch = [float(m.group(1)) for l in lines for m in [re.match(r"krk_engine sha t=\S+ abs=([\d.]+)ms", l)] if m]
for r in rounds:
    go, end = r["t_go_ms"], r["t_go_ms"] + 1e3 * r["seconds"]
    s = [x for x in slow if go - 1 <= x[2] <= end]
    L = [x for x in launch if go - 1 <= x <= end]
    c = collections.Counter(x[0] for x in s)
    worst = sorted(s, key=lambda x: -x[1])[:3]
    print(f"round {r['round']}: {r['GBps']} GB/s; slow steps {dict(c)}; worst "
          f"{[(w[0], round(w[1], 1), round(w[2] - go, 1)) for w in worst]}; launches at "
          f"{[round(x - go, 1) for x in L[:3]]}")
