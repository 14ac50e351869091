"""VALU / LDS utilisation per kernel from rocprofv3 PMC passes -> profiles/r02/valu_<workload>.json.

Each pass is its own run with only --kernel-trace beside --pmc (tools/gpu_round.sh
`valu` / `value2e`), e.g.

  rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \\
      SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv -d DIR -- python3 bench.py ...

Units (MI355X_MICROARCH.md, per-instruction constants table): SQ_WAVE_CYCLES,
SQ_BUSY_CYCLES, SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles (4 shader cycles);
GRBM_GUI_ACTIVE counts cycles summed over the 8 XCDs.  Reported per kernel, summed
over its dispatches in the profiled run:

  valu_issue_frac_per_wave = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
        the fraction of its lifetime an average wave of the kernel spends issuing
        VALU (a wave alone issues one VALU per 4-cycle quad at best)
  valu_busy_chip_pct = 100 * 4 * SQ_ACTIVE_INST_VALU / (SIMDs * GRBM_GUI_ACTIVE / 8)
        VALU issue cycles over every SIMD-cycle of the kernel's run (rocprof's
        VALUBusy form): low when few SIMDs hold the kernel's waves
  lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles over
        all LDS-array cycles)
  clock_mhz = GRBM_GUI_ACTIVE / 8 / summed kernel time (trustworthy for dispatches
        longer than ~0.3 ms)
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

KERNELS = {"crc_items_kernel": "crc32_pieces", "gather_kernel": "host_gather", "sha256_ws_kernel": "sha256_multi", "sha256_w8_kernel": "sha256_multi",
           "hrw_order_kernel": "hrw_order",
           "shard_gather_kernel": "hrw_gather", "shard_gather_packed_kernel": "hrw_gather",
           "pack_owner_rows_kernel": "hrw_order", "synth_fill": "synth_fill"}
SIMDS = 1024  # 256 CUs x 4 SIMD-32


def _short(name):
    for k, v in sorted(KERNELS.items(), key=lambda kv: -len(kv[0])):  # the longest name first
        if k in name:
            return v
    return None


def read_dir(d, longest=False):
    """({kernel: {counter: total}}, {kernel: [dispatches, total ns]}); longest: only each
    kernel's longest dispatch (the workload's own launch when the run has shorter ones of the
    same kernel: calibration, a host-offload leg's prefixes)."""
    dur = {}  # dispatch id -> (kernel, ns)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = _short(row.get("Kernel_Name", ""))
                if k:
                    dur[row.get("Dispatch_Id") or row.get("Correlation_Id")] = (
                        k, int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    keep = None
    if longest:
        best = {}
        for did, (k, ns) in dur.items():
            if k not in best or ns > best[k][1]:
                best[k] = (did, ns)
        keep = {did for did, _ in best.values()}
    ctr = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = _short(row.get("Kernel_Name", ""))
                did = row.get("Dispatch_Id") or row.get("Correlation_Id")
                if k and (keep is None or did in keep):
                    ctr[k][row["Counter_Name"]] += float(row["Counter_Value"])
    tim = defaultdict(lambda: [0, 0])
    for did, (k, ns) in dur.items():
        if keep is None or did in keep:
            tim[k][0] += 1
            tim[k][1] += ns
    return ctr, tim


def metrics(c, t):
    g = lambda k: c.get(k)  # noqa: E731
    out = {"counters": dict(c), "dispatches": t[0], "kernel_ms": round(t[1] / 1e6, 3)}
    if g("SQ_ACTIVE_INST_VALU") and g("SQ_WAVE_CYCLES"):
        out["valu_issue_frac_per_wave"] = round(g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES"), 4)
    if g("SQ_ACTIVE_INST_VALU") and g("GRBM_GUI_ACTIVE"):
        out["valu_busy_chip_pct"] = round(100 * 4 * g("SQ_ACTIVE_INST_VALU") / (SIMDS * g("GRBM_GUI_ACTIVE") / 8), 3)
    if g("SQ_ACTIVE_INST_LDS") and g("SQ_WAVE_CYCLES"):
        out["lds_issue_frac_per_wave"] = round(g("SQ_ACTIVE_INST_LDS") / g("SQ_WAVE_CYCLES"), 4)
    if g("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_frac"] = round((g("SQ_LDS_BANK_CONFLICT") or 0.0) / g("SQ_LDS_IDX_ACTIVE"), 4)
    if g("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if g(k) is not None:
                out[k.lower()[3:] + "_frac_per_wave"] = round(g(k) / g("SQ_WAVE_CYCLES"), 4)
    if g("GRBM_GUI_ACTIVE") and t[1]:
        out["clock_mhz"] = round(g("GRBM_GUI_ACTIVE") / 8 / (t[1] / 1e3), 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dirs", nargs="+", required=True, help="rocprofv3 output dirs (one per counter pass)")
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--mode", default="device_resident", choices=["device_resident", "end_to_end"])
    ap.add_argument("--what", default="")
    ap.add_argument("--out", default=None)
    ap.add_argument("--longest", action="store_true", help="only each kernel's longest dispatch")
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = a.out or os.path.join(root, "profiles", "r02", f"valu_{a.workload}.json")
    ctr = defaultdict(dict)
    tim = {}
    for d in a.dirs:
        c, t = read_dir(d, a.longest)
        for k, v in c.items():
            ctr[k].update(v)
        for k, v in t.items():
            tim[k] = v  # every pass runs the same command: keep one pass's trace
    try:
        res = json.load(open(out))
    except (OSError, ValueError):
        res = {"workload": a.workload, "definitions": __doc__.split("Units")[1].strip()}
    res[a.mode] = {k: metrics(v, tim.get(k, [0, 0])) for k, v in sorted(ctr.items())}
    if a.what:
        res[a.mode]["what"] = a.what
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res[a.mode], indent=1))


if __name__ == "__main__":
    main()
