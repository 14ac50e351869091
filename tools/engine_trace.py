"""Per-round timeline of the native digester harness under KRK_ENGINE_TRACE=1:
go -> first launch, launch cadence, gaps, last retire -> round end.
    python tools/engine_trace.py gpurun_out/nd_trace.log"""
import json
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
rounds = [json.loads(l) for l in lines if l.startswith("{")]
ev = []
for l in lines:
    m = re.match(r"krk_engine sha t=\S+ abs=([\d.]+)ms n=(\d+) why=(\S)", l)
    if m:
        ev.append(("L", float(m.group(1)), int(m.group(2)), m.group(3)))
    m = re.match(r"krk_engine sha_done abs=([\d.]+)ms n=(\d+)", l)
    if m:
        ev.append(("D", float(m.group(1)), int(m.group(2)), ""))
for r in rounds:
    go, end = r["t_go_ms"], r["t_go_ms"] + 1e3 * r["seconds"]
    e = [x for x in ev if go - 1 <= x[1] <= end + 1]
    L = [x for x in e if x[0] == "L"]
    Dn = [x for x in e if x[0] == "D"]
    if not L:
        continue
    gaps = [round(b[1] - a[1], 1) for a, b in zip(Dn, Dn[1:]) if b[1] - a[1] > 12]
    print(f"round {r['round']}: {r['GBps']} GB/s, {r['seconds']*1e3:.1f} ms; go->1st launch {L[0][1]-go:.1f} ms "
          f"(n={L[0][2]} why={L[0][3]}); 1st->last retire {Dn[-1][1]-L[0][1]:.1f} ms over {len(L)} launches; "
          f"last retire->end {end-Dn[-1][1]:.1f} ms; retire gaps >12 ms: {gaps}; small launches: "
          f"{[x[2] for x in L if x[2] < 240]}")
