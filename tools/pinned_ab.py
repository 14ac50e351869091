"""A/B of the pinned-source path of krk_metainfo_digest_host: blobs in
page-locked host memory (krk_host_alloc), windows of <= 64 chunks DMA'd straight from the
caller's pages (KRK_PINNED_DIRECT=1, the default) against the same windows staged through
the pinned window by host copies (KRK_PINNED_DIRECT=0).  Each leg runs in its own process
(the switch is read once); host offload off, so every byte crosses the link.

    python tools/pinned_ab.py [blobs] [MiB each]      one JSON line per leg"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LEG = r"""
import json, sys, time
import numpy as np
sys.path.insert(0, %(root)r)
from kraken_amd import device as D
n, mib = %(n)d, %(mib)d
L = mib << 20
D.set_sha_host_offload(0)
bufs = []
for i in range(n):
    pa = D.PinnedArray((L,), np.uint8)
    dev = D.DeviceBuffer(L)
    D.check(D.lib.krk_synth_fill_dev(dev.ptr, (5 << 40) + i, 0, L, 0, None))
    D.synchronize()
    D.check(D.lib.krk_memcpy_d2h(pa.a.ctypes.data, dev.ptr, L))
    dev.free()
    bufs.append(pa)
datas = [b.a for b in bufs]
D.metainfo_digest_host(datas, 4 << 20)  # warm
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    sums, dg = D.metainfo_digest_host(datas, 4 << 20)
    ts.append(time.perf_counter() - t0)
st = D.windows_last_call()
el = float(np.median(ts))
print(json.dumps({"direct_env": %(direct)r, "blobs": n, "bytes_each": L, "GBps": round(n * L / el / 1e9, 3),
                  "passes_s": [round(x, 3) for x in ts], "windows": st,
                  "digest0": bytes(dg[0]).hex(), "digest_last": bytes(dg[-1]).hex()}))
"""


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 48
    mib = int(sys.argv[2]) if len(sys.argv) > 2 else 192
    out = []
    for direct in ("1", "0"):
        env = dict(os.environ, KRK_PINNED_DIRECT=direct)
        r = subprocess.run([sys.executable, "-c", LEG % dict(root=ROOT, n=n, mib=mib, direct=direct)], env=env,
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            print(r.stderr[-3000:], file=sys.stderr)
            return r.returncode
        line = json.loads(r.stdout.strip().splitlines()[-1])
        out.append(line)
        print(json.dumps(line), flush=True)
    same = out[0]["digest0"] == out[1]["digest0"] and out[0]["digest_last"] == out[1]["digest_last"]
    print(json.dumps({"digests_equal": same, "direct_over_staged": round(out[0]["GBps"] / out[1]["GBps"], 3)}))
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
