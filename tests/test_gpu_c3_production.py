"""Config C3 in its production launch shape (kraken_amd.windowed, what bench.py's C3
line runs), at a scaled size whose one-shot results fit in HBM.

16,384 blobs drawn from the C3 length law (100 MiB + rng mod
968,884,225 B) with every length divided by 64 (1.6-16.7 MB, byte-granular, so most
blobs end in a partial 4 MiB piece).  With the planner's own live cap
(window_stream_cap: 7/8 of the two-lane stream count, 14,336 on 256 CUs) the first
windows run 14,336 live streams: two lanes a stream, two producer/consumer pairs a
workgroup (KRK_SHA_PLAN_2LANE_2PAIR), 224 SHA workgroups on 224 CUs, and each
window's piece-CRC launch on the 32 CUs left free, in flight together with the SHA
launch.  2,048 blobs wait and are admitted as earlier ones finish.

Every blob's digest and piece sums are compared with the one-shot device path
(krk_metainfo_digest_dev, in batches), and the shortest, the longest, a
partial-last-piece blob and a late-admitted blob with hashlib / the oracle
(core/metainfo.go:157-179, core/digester.go:41-72).  The same check runs on rank 0's
LPT shard of an 8-GPU split (bench.py --emulate-world 8): ~2,000 blobs on the
eight-lane plan."""
import hashlib

import numpy as np
import pytest

from kraken_amd import device as D
from kraken_amd.shard import lpt_shard
from kraken_amd.windowed import WindowedRun, c3_lengths, two_lane_stream_cap, window_stream_cap

pytestmark = pytest.mark.gpu

N, SCALE, P = 16384, 64, 4 << 20
W = 16 << 30  # window bytes: 10 windows for the scaled batch, the first 5 with 14,336 live
BATCH = 4096  # one-shot reference batch (blobs): ~38 GB of arena at a time


@pytest.fixture(scope="module")
def c3_scaled(gpu):
    lens = c3_lengths(N, scale=SCALE)
    ids = [(2 << 40) + i for i in range(N)]
    dg = np.zeros((N, 32), dtype=np.uint8)
    sums = {}
    for b0 in range(0, N, BATCH):
        sl = slice(b0, min(N, b0 + BATCH))
        arena = D.BlobArena(lens[sl], P, blob_ids=ids[sl])
        out = D.BatchOutputs(arena)
        D.metainfo_digest(arena, out)
        D.synchronize()
        dg[sl] = out.digests.to_host(np.uint8, 32 * (sl.stop - sl.start)).reshape(-1, 32)
        s = out.sums.to_host(np.uint32, arena.total_pieces)
        for k in range(sl.stop - sl.start):
            o, c = int(arena.sums_off[k]), int(arena.n_pieces[k])
            sums[b0 + k] = s[o:o + c].copy()
        del arena, out
    return lens, ids, dg, sums


def _run_windowed(lens, ids):
    wr = WindowedRun(D, ids, lens, P, W)
    with D.KernelTimer():
        wr.run()
        sha = D.KernelTimer.timeline("sha256_multi")
        crc = D.KernelTimer.timeline("crc32_pieces")
    cb = wr.cb
    n = len(lens)
    dg = cb.digests.to_host(np.uint8, 32 * n).reshape(-1, 32)
    s = cb.sums.to_host(np.uint32, max(cb.total_pieces, 1))
    sums = [s[int(cb.sums_off[i]):int(cb.sums_off[i]) + int(cb.n_pieces[i])] for i in range(n)]
    wins, cap = wr.wins, wr.cap
    wr.close()
    return dg, sums, wins, cap, sha, crc


def _check_oracle(orc, lens, ids, dg, sums, picks):
    for i in picks:
        data = orc.synth(ids[i], lens[i])
        assert bytes(dg[i]) == hashlib.sha256(data.tobytes()).digest(), i
        assert np.array_equal(sums[i], orc.calc_piece_sums(data, P)[1]), i


def test_c3_production_window_shape_two_lane_two_pair(c3_scaled, orc):
    lens, ids, dg1, sums1 = c3_scaled
    cus = two_lane_stream_cap(D, 1 << 30) // 64  # the two-lane plan holds 64 streams a CU
    dg, sums, wins, cap, sha, crc = _run_windowed(lens, ids)

    # the planner's cap, not a test override: 7/8 of the two-lane stream count
    assert cap == window_stream_cap(D, N) == (64 * cus * 7 // 8) // 64 * 64
    assert D.sha_plan_for(cap) == 4, D.SHA_PLAN_NAMES.get(D.sha_plan_for(cap))  # KRK_SHA_PLAN_2LANE_2PAIR
    assert D.sha_lanes_per_stream(cap) == 2
    assert len(wins[0][0]) == cap < N and len(wins) > 8
    # what the launches actually ran: the first windows' SHA launches carry `cap`
    # streams on the two-lane two-pair plan; 64 streams per 2-pair workgroup leave
    # cus - cap / 64 CUs without a SHA workgroup for the window's CRC launch
    assert len(sha) == len(wins) and len(crc) == len(wins)
    full = [k for k, w in enumerate(wins) if len(w[0]) == cap]
    assert len(full) >= 3
    for k in full:
        plan, units, s0, s1 = sha[k]
        assert plan == 4 and units == cap, (k, plan, units)
        c0, c1 = crc[k][2], crc[k][3]
        assert c0 < s1 and c1 > s0, (k, (s0, s1), (c0, c1))  # the CRC launch was in flight with the SHA launch
    assert cus - cap // 64 >= cus // 8
    # late admission happened: some blobs first appear after window 0
    first = {}
    for k, (blobs, offs, take) in enumerate(wins):
        for b in blobs[offs == 0]:
            first.setdefault(int(b), k)
    late = sorted(b for b, k in first.items() if k > 0)
    assert len(late) == N - cap

    # every blob equal to the one-shot path
    assert np.array_equal(dg, dg1)
    for i in range(N):
        assert np.array_equal(sums[i], sums1[i]), i
    L = np.asarray(lens)
    partial = int(np.flatnonzero(L % P)[0])
    _check_oracle(orc, lens, ids, dg, sums, sorted({int(L.argmin()), int(L.argmax()), partial, late[-1]}))


def test_c3_emulated_world8_shard(c3_scaled, orc):
    """bench.py --emulate-world 8 at scaled size: rank 0's LPT shard alone through the
    windowed path -- the eight-lane plan (<= 16 x CUs live streams)."""
    lens, ids, dg1, sums1 = c3_scaled
    mine = lpt_shard(lens, 8)[0]
    ls, ii = [lens[i] for i in mine], [ids[i] for i in mine]
    dg, sums, wins, cap, sha, crc = _run_windowed(ls, ii)
    cus = two_lane_stream_cap(D, 1 << 30) // 64
    assert cap == len(mine) <= 16 * cus
    assert D.sha_plan_for(len(mine)) == 5 and sha[0][0] == 5 and sha[0][1] == len(mine)  # KRK_SHA_PLAN_8LANE
    assert max(ls) == max(lens)  # LPT gives rank 0 the longest blob
    for k, i in enumerate(mine):
        assert bytes(dg[k]) == bytes(dg1[i]), i
        assert np.array_equal(sums[k], sums1[i]), i
    L = np.asarray(ls)
    _check_oracle(orc, ls, ii, dg, sums, sorted({int(L.argmin()), int(L.argmax())}))
