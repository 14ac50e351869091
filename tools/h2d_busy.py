"""H2D link occupancy of a windowed host pass from a rocprofv3 --memory-copy-trace CSV:
the staging windows' uploads (copies > 5 ms) grouped into passes (a gap > 50 ms starts a
new group), each group's wall time, summed copy time, busy fraction and per-copy rate.

  python tools/h2d_busy.py gpurun_out/prof_e2e [window MiB]"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    win = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    f = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    big = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                 if r["Direction"] == "MEMORY_COPY_HOST_TO_DEVICE"
                 and int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 5_000_000)
    groups, cur = [], [big[0]]
    for x in big[1:]:
        if x[0] - cur[-1][1] > 50_000_000:
            groups.append(cur)
            cur = [x]
        else:
            cur.append(x)
    groups.append(cur)
    for g in groups:
        wall = (g[-1][1] - g[0][0]) / 1e9
        busy = sum(b - a for a, b in g) / 1e9
        gaps = [g[i + 1][0] - g[i][1] for i in range(len(g) - 1)]
        print(f"uploads={len(g)} wall={wall:.3f}s h2d_busy={busy:.3f}s busy_frac={busy / wall:.3f} "
              f"mean_gap_ms={sum(gaps) / max(1, len(gaps)) / 1e6:.3f} max_gap_ms={(max(gaps) if gaps else 0) / 1e6:.2f} "
              f"GBps_per_copy={(win << 20) / (busy / len(g)) / 1e9:.1f}")


if __name__ == "__main__":
    main()
