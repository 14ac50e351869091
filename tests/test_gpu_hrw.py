"""GPU parity: lib/hrw scores/orders and hashring Locations through the C ABI vs
the CPU oracle.  Scores must match bit for bit (fp64, Go math.Log restated, no
FMA).  Distribution properties follow lib/hrw/rendezvous_test.go:100-274."""
import os

import numpy as np
import pytest

from kraken_amd import hashring, hrw
from kraken_amd import device as D
from kraken_amd._capi import check, lib

pytestmark = pytest.mark.gpu


def _keys(rng, n, nbytes):
    return [rng.bytes(nbytes).hex() for _ in range(n)]


@pytest.mark.parametrize("n_nodes", [1, 3, 5, 16, 64])
@pytest.mark.parametrize("weighted", [False, True])
def test_scores_and_orders_match_oracle(gpu, orc, n_nodes, weighted):
    rng = np.random.default_rng(n_nodes * 2 + weighted)
    labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(n_nodes)]
    weights = [[100, 200, 400, 800][i % 4] if weighted else 100 for i in range(n_nodes)]
    rh = hrw.NewRendezvousHash()
    for l, w in zip(labels, weights):
        rh.AddNode(l, w)
    keys = _keys(rng, 300, 2) + _keys(rng, 100, 1) + _keys(rng, 100, 32) + _keys(rng, 50, 64)
    order = rh.GetOrderedNodesBatch(keys, n_nodes)
    scores = rh.Scores(keys)
    for i, k in enumerate(keys):
        ref_o, ref_s = orc.hrw_ordered(k, labels, weights, with_scores=True)
        assert order[i].tolist() == ref_o, k
        assert scores[i].tobytes() == np.asarray(ref_s, dtype=np.float64).tobytes(), k


def test_survey_sanity_vector(gpu):
    """dummy-origin-master0{1,2,3}-zone2:80, weight 100."""
    rh = hrw.NewRendezvousHash()
    for i in (1, 2, 3):
        rh.AddNode(f"dummy-origin-master0{i}-zone2:80", 100)
    lab = lambda k: [n.Label[len("dummy-origin-master0")] for n in rh.GetOrderedNodes(k, 3)]
    assert lab("e3b0") == ["3", "2", "1"]
    assert lab("0000") == ["1", "3", "2"]
    assert lab("ffff") == ["1", "3", "2"]


def test_get_ordered_nodes_n_and_invalid_hex(gpu):
    rh = hrw.NewRendezvousHash()
    for i, w in enumerate([100, 200, 400, 800]):
        rh.AddNode(str(i), w)
    assert len(rh.GetOrderedNodes("abcd", 2)) == 2
    assert len(rh.GetOrderedNodes("abcd", 10)) == 4
    assert np.isnan(rh.Nodes[0].Score("zz"))  # rendezvous.go:154-157
    assert [n.Label for n in rh.GetOrderedNodes("xyz", 4)] == ["0", "1", "2", "3"]


def test_key_distribution_weighted(gpu):
    """rendezvous_test.go:145-148: keys split ~ weights 100/200/400/800 (+-0.1)."""
    rh = hrw.NewRendezvousHash()
    ws = [100, 200, 400, 800]
    for i, w in enumerate(ws):
        rh.AddNode(str(i), w)
    rng = np.random.default_rng(0)
    keys = _keys(rng, 20000, 64)
    first = rh.GetOrderedNodesBatch(keys, 1)[:, 0]
    frac = np.bincount(first, minlength=4) / len(keys)
    assert np.all(np.abs(frac - np.array(ws) / 1500.0) < 0.1 * np.array(ws) / 1500.0 + 0.01), frac


def test_add_remove_node_stability(gpu):
    """rendezvous_test.go:150-193: removing a node only moves its own keys."""
    rh = hrw.NewRendezvousHash()
    for i, w in enumerate([100, 200, 400, 800]):
        rh.AddNode(str(i), w)
    rng = np.random.default_rng(9)
    keys = _keys(rng, 5000, 32)
    before = [rh.Nodes[j].Label for j in rh.GetOrderedNodesBatch(keys, 1)[:, 0]]
    rh.RemoveNode("1")
    after = [rh.Nodes[j].Label for j in rh.GetOrderedNodesBatch(keys, 1)[:, 0]]
    for b, a in zip(before, after):
        if b != "1":
            assert a == b


@pytest.mark.parametrize("n_nodes,max_replica", [(3, 3), (5, 2), (16, 3), (64, 2), (4, 0), (4, 10)])
def test_ring_locations_match_oracle(gpu, orc, n_nodes, max_replica):
    rng = np.random.default_rng(n_nodes + 31 * max_replica)
    labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(n_nodes)]
    for healthy in (np.ones(n_nodes, np.uint8), (rng.random(n_nodes) < 0.75).astype(np.uint8),
                    np.zeros(n_nodes, np.uint8)):
        ring = hashring.Ring(labels, [l for l, h in zip(labels, healthy) if h], max_replica)
        digests = rng.integers(0, 256, size=(2000, 32), dtype=np.uint8)
        locs, counts = ring.LocationsBatch(digests)
        for i in range(len(digests)):
            key = bytes(digests[i, :2]).hex()
            order = orc.hrw_ordered(key, labels, [100] * n_nodes)
            ref = orc.ring_locations(order, healthy, max_replica)
            assert locs[i, : counts[i]].tolist() == ref, (i, key)


def test_ring_locations_dev_full_table(gpu, orc):
    """Device-resident 65,536-shard table + gather (config C5 path) vs oracle."""
    n_nodes, max_replica = 16, 3
    labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(n_nodes)]
    rng = np.random.default_rng(77)
    healthy = (rng.random(n_nodes) < 0.75).astype(np.uint8)
    n = 50000
    digests = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    dbuf = D.DeviceBuffer(n * 32)
    dbuf.from_host(digests.reshape(-1))
    lbuf = D.DeviceBuffer(n * max_replica * 4)
    cbuf = D.DeviceBuffer(n)
    D.ring_locations_dev(dbuf, n, labels, healthy, max_replica, lbuf, cbuf)
    D.synchronize()
    locs = lbuf.to_host(np.int32, n * max_replica).reshape(n, max_replica)
    counts = cbuf.to_host(np.uint8, n)
    cache = {}
    for i in range(0, n, 7):
        key = bytes(digests[i, :2]).hex()
        if key not in cache:
            cache[key] = orc.ring_locations(orc.hrw_ordered(key, labels, [100] * n_nodes), healthy, max_replica)
        assert locs[i, : counts[i]].tolist() == cache[key]
    ring = hashring.Ring(labels, [l for l, h in zip(labels, healthy) if h], max_replica)
    from kraken_amd import core
    d = core.NewSHA256DigestFromHex(bytes(digests[0]).hex())
    assert ring.Locations(d) == [labels[j] for j in locs[0, : counts[0]]]


def test_ring_owner_tables_cached_by_membership(gpu, orc):
    """Owner tables are kept per membership (ring.Refresh semantics, lib/hashring/ring.go:
    141-165): twelve memberships (more than the eight a device keeps) visited twice in
    interleaved order -- hits, misses and evictions -- every result against the oracle,
    including a health flip that keeps the labels and a relabelled node."""
    rng = np.random.default_rng(0x0C5)
    n = 4096
    digests = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    dbuf = D.DeviceBuffer(n * 32)
    dbuf.from_host(digests.reshape(-1))
    rings = []
    for k in range(12):
        N = [3, 5, 16, 64][k % 4]
        labels = [f"origin-{i:03d}.kraken.test:{15002 + (k // 4)}" for i in range(N)]
        healthy = (rng.random(N) < 0.75).astype(np.uint8)
        rings.append((labels, healthy, 2 + k % 2))
    labels, healthy, R = rings[0]
    flipped = healthy.copy()
    flipped[0] ^= 1
    rings.append((labels, flipped, R))  # same labels, other health: its own table
    rings.append((labels[:-1] + ["origin-zzz.kraken.test:15002"], healthy, R))
    lbuf = D.DeviceBuffer(n * 3)
    cbuf = D.DeviceBuffer(n)
    picks = list(range(0, n, 97))
    for rep in range(2):
        for labels, healthy, R in (rings if rep == 0 else rings[::-1]):
            D.ring_locations_u8_dev(dbuf, n, labels, healthy, R, lbuf, cbuf)
            D.synchronize()
            locs = lbuf.to_host(np.uint8, n * R).reshape(n, R)
            counts = cbuf.to_host(np.uint8, n)
            N = len(labels)
            for i in picks:
                key = bytes(digests[i, :2]).hex()
                want = orc.ring_locations(orc.hrw_ordered(key, labels, [100] * N), healthy, R)
                assert locs[i, : counts[i]].tolist() == want, (rep, N, R, i)


def test_ring_owner_tables_concurrent_callers_with_evictions(gpu):
    """ADVICE r05 (owner-table slots): eight threads place digests over twelve memberships at
    once (more than the eight tables a device keeps), so tables are built, used and evicted
    while other callers' launches still read theirs.  A table in use is never evicted and a
    failed or replaced build never moves another caller's slot: every thread's owner lists
    equal the serial run's for that membership, every time."""
    import threading
    rng = np.random.default_rng(0xC0C5)
    n = 8192
    digests = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    dbuf = D.DeviceBuffer(n * 32)
    dbuf.from_host(digests.reshape(-1))
    rings = []
    for k in range(12):
        N = [3, 5, 16, 64][k % 4]
        labels = [f"origin-{i:03d}.kraken.test:{16002 + k}" for i in range(N)]
        rings.append((labels, (rng.random(N) < 0.8).astype(np.uint8), 2 + k % 2))
    want = []
    lb, cb = D.DeviceBuffer(n * 3), D.DeviceBuffer(n)
    for labels, healthy, R in rings:  # serial
        D.ring_locations_u8_dev(dbuf, n, labels, healthy, R, lb, cb)
        D.synchronize()
        want.append((lb.to_host(np.uint8, n * R).copy(), cb.to_host(np.uint8, n).copy()))
    errors = []

    def caller(t):
        try:
            D.set_device(0)
            r = np.random.default_rng(t)
            mlb, mcb = D.DeviceBuffer(n * 3), D.DeviceBuffer(n)
            for _ in range(30):
                k = int(r.integers(0, len(rings)))
                labels, healthy, R = rings[k]
                D.ring_locations_u8_dev(dbuf, n, labels, healthy, R, mlb, mcb)
                D.synchronize()
                got = (mlb.to_host(np.uint8, n * R), mcb.to_host(np.uint8, n))
                if not (np.array_equal(got[0], want[k][0]) and np.array_equal(got[1], want[k][1])):
                    errors.append((t, k))
        except Exception as e:  # surfaced below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=caller, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not any(x.is_alive() for x in th)
    assert not errors, errors[:5]


def test_cas_volume_placement(gpu, orc, tmp_path):
    """lib/store/ca_store.go:137-171: weighted HRW over volumes for subdirs "%02X"."""
    from kraken_amd import castore
    vols = []
    for i, w in enumerate((100, 200, 400, 800)):
        p = tmp_path / f"vol{i}"
        p.mkdir()
        vols.append(castore.Volume(str(p), w))
    m = castore.volume_subdirs(vols)
    labels, weights = [v.Location for v in vols], [v.Weight for v in vols]
    for sub, loc in m.items():
        assert loc == labels[orc.hrw_ordered(sub, labels, weights)[0]], sub
    d = tmp_path / "cas"
    d.mkdir()
    castore.initCASVolumes(str(d), vols)
    for sub, loc in m.items():
        assert os.readlink(d / sub) == os.path.join(loc, "cas", sub)
        assert (d / sub).is_dir()
    castore.initCASVolumes(str(d), vols)  # idempotent
    with pytest.raises(OSError, match="verify volume"):
        castore.initCASVolumes(str(d), [castore.Volume(str(tmp_path / "missing"), 100)])


@pytest.mark.gpu
@pytest.mark.parametrize("n_nodes,max_replica", [(16, 3), (255, 2), (5, 8)])
def test_ring_locations_u8_dev_equals_int32_path(gpu, orc, n_nodes, max_replica):
    """krk_ring_locations_u8_dev: the same owner lists as the int32 path (0xFF where it
    pads -1), counts identical; spot rows against the oracle."""
    labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(n_nodes)]
    rng = np.random.default_rng(1000 + n_nodes)
    healthy = (rng.random(n_nodes) < 0.75).astype(np.uint8)
    n = 30001
    digests = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    dbuf = D.DeviceBuffer(n * 32)
    dbuf.from_host(digests.reshape(-1))
    l32, c32 = D.DeviceBuffer(n * max_replica * 4), D.DeviceBuffer(n)
    l8, c8 = D.DeviceBuffer(n * max_replica), D.DeviceBuffer(n)
    D.ring_locations_dev(dbuf, n, labels, healthy, max_replica, l32, c32)
    D.ring_locations_u8_dev(dbuf, n, labels, healthy, max_replica, l8, c8)
    D.synchronize()
    a32 = l32.to_host(np.int32, n * max_replica).reshape(n, max_replica)
    a8 = l8.to_host(np.uint8, n * max_replica).reshape(n, max_replica)
    assert np.array_equal(np.where(a32 < 0, 255, a32).astype(np.uint8), a8)
    assert np.array_equal(c32.to_host(np.uint8, n), c8.to_host(np.uint8, n))
    for i in range(0, n, 997):
        key = bytes(digests[i, :2]).hex()
        want = orc.ring_locations(orc.hrw_ordered(key, labels, [100] * n_nodes), healthy, max_replica)
        assert a8[i, : len(want)].tolist() == want


@pytest.mark.gpu
@pytest.mark.parametrize("max_replica", [1, 2, 3, 5])
def test_ring_locations_u8_dev_offsets_and_tails(gpu, max_replica):
    """Compact owner lists at any output address and count: word-aligned outputs take the
    packed-row gather (four digests a thread, word stores, rows of <= 3), others and rows
    of more owners the byte-store gather; every layout and every tail length gives the
    int32 path's lists."""
    import ctypes as C
    labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(16)]
    healthy = np.ones(16, dtype=np.uint8)
    healthy[[2, 9]] = 0
    rng = np.random.default_rng(77 + max_replica)
    for n in (1, 3, 4, 5, 1023, 4097):
        digests = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        dbuf = D.DeviceBuffer(n * 32)
        dbuf.from_host(digests.reshape(-1))
        l32, c32 = D.DeviceBuffer(n * max_replica * 4), D.DeviceBuffer(n)
        D.ring_locations_dev(dbuf, n, labels, healthy, max_replica, l32, c32)
        D.synchronize()
        want = np.where(l32.to_host(np.int32, n * max_replica) < 0, 255,
                        l32.to_host(np.int32, n * max_replica)).astype(np.uint8)
        wc = c32.to_host(np.uint8, n)
        for shift, cshift in ((0, 0), (1, 1), (3, 3), (0, 2), (4, 0)):
            lb, cb = D.DeviceBuffer(n * max_replica + 8), D.DeviceBuffer(n + 8)
            s, keep = D.nodes_struct(labels, [100] * 16)
            check(lib.krk_ring_locations_u8_dev(dbuf.ptr, n, C.byref(s), healthy.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                 max_replica, lb.ptr + shift, cb.ptr + cshift, None))
            D.synchronize()
            assert np.array_equal(lb.to_host(np.uint8, n * max_replica, shift), want), (n, shift)
            assert np.array_equal(cb.to_host(np.uint8, n, cshift), wc), (n, cshift)
        # a digest array at an odd address (byte loads) and at a 2-byte one (16-bit loads)
        for dshift in (1, 2):
            db2 = D.DeviceBuffer(n * 32 + 4)
            db2.from_host(np.concatenate([np.zeros(dshift, np.uint8), digests.reshape(-1)]))
            lb, cb = D.DeviceBuffer(n * max_replica), D.DeviceBuffer(n)
            s, keep = D.nodes_struct(labels, [100] * 16)
            check(lib.krk_ring_locations_u8_dev(db2.ptr + dshift, n, C.byref(s),
                                                 healthy.ctypes.data_as(C.POINTER(C.c_uint8)), max_replica, lb.ptr,
                                                 cb.ptr, None))
            D.synchronize()
            assert np.array_equal(lb.to_host(np.uint8, n * max_replica), want), (n, dshift)
            assert np.array_equal(cb.to_host(np.uint8, n), wc), (n, dshift)


@pytest.mark.gpu
def test_ring_locations_u8_dev_rejects_256_nodes(gpu):
    labels = [f"o{i}" for i in range(256)]
    dbuf, lb, cb = D.DeviceBuffer(32), D.DeviceBuffer(3), D.DeviceBuffer(1)
    with pytest.raises(Exception, match="255"):
        D.ring_locations_u8_dev(dbuf, 1, labels, np.ones(256, np.uint8), 3, lb, cb)


def _u64_to_f64_dev(vals, rehash):
    import ctypes as C
    from kraken_amd._capi import check, lib
    be = np.array(vals, dtype=">u8").view(np.uint8)
    out = np.zeros(len(vals), dtype=np.float64)
    check(lib.krk_hrw_uint64_to_float64(be.ctypes.data_as(C.POINTER(C.c_uint8)), len(vals), int(rehash),
                                        out.ctypes.data_as(C.POINTER(C.c_double))))
    return out


def test_uint64_to_float64_rehash_branch_on_device(gpu, orc):
    """lib/hrw/rendezvous_test.go:59-98 (TestScoreFunctionUint64ToFloat64BadValues): the
    12 Sum values 2^53 .. 2^64 (the last wraps to 0 in Go's int) have all-zero low 53
    bits.  With a nil hasher the score is 0.0; with murmur3 it is re-hashed once and is
    non-zero with a finite log -- through the scoring kernel's own device function, bit
    for bit against the oracle.  Random Sums (no rehash) must match too."""
    vals = [((1 << 53) << i) & ((1 << 64) - 1) for i in range(12)]
    assert all(v & ((1 << 53) - 1) == 0 for v in vals)
    nil = _u64_to_f64_dev(vals, False)
    assert (nil == 0.0).all()
    got = _u64_to_f64_dev(vals, True)
    for v, g in zip(vals, got):
        want = orc.uint64_to_float64(v, True)
        assert g.tobytes() == np.float64(want).tobytes(), hex(v)
        assert g != 0.0 and np.isfinite(np.log(g))
        assert np.isfinite(orc.go_log(float(g)))
    rng = np.random.default_rng(53)
    rnd = [int(x) for x in rng.integers(0, 2 ** 63, 4096, dtype=np.int64)] + [0, (1 << 64) - 1, (1 << 53) - 1]
    got = _u64_to_f64_dev(rnd, True)
    for v, g in zip(rnd, got):
        assert g.tobytes() == np.float64(orc.uint64_to_float64(v, True)).tobytes(), hex(v)


@pytest.mark.parametrize("n_nodes,max_replica", [(3, 2), (16, 3), (64, 2)])
def test_ring_owner_table_lookup(gpu, orc, n_nodes, max_replica):
    """Ring.Refresh builds all 65,536 owner lists (krk_ring_owner_table); Locations is a
    host lookup of the ShardID row.  Every 97th row against the oracle, the lookups
    against the per-call path, and a health change followed by Refresh."""
    from kraken_amd import core
    rng = np.random.default_rng(n_nodes * 7 + max_replica)
    labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(n_nodes)]
    healthy = (rng.random(n_nodes) < 0.75).astype(np.uint8)
    healthy[0] = 1
    ring = hashring.Ring(labels, [l for l, h in zip(labels, healthy) if h], max_replica)
    ring.Refresh()
    locs, counts = ring._table
    assert locs.shape == (65536, max(1, max_replica))
    for shard in range(0, 65536, 97):
        key = f"{shard:04x}"
        ref = orc.ring_locations(orc.hrw_ordered(key, labels, [100] * n_nodes), healthy, max_replica)
        assert locs[shard, : counts[shard]].tolist() == ref, key
    digests = rng.integers(0, 256, size=(500, 32), dtype=np.uint8)
    bl, bc = ring.LocationsBatch(digests)
    for i in range(len(digests)):
        d = core.NewSHA256DigestFromHex(bytes(digests[i]).hex())
        assert ring.Locations(d) == [labels[j] for j in bl[i, : bc[i]]]
    ring.set_healthy([])  # all unhealthy: [order[0]] per shard
    d = core.NewSHA256DigestFromHex(bytes(digests[0]).hex())
    key = d.ShardID()
    assert ring.Locations(d) == [labels[orc.hrw_ordered(key, labels, [100] * n_nodes)[0]]]


@pytest.mark.gpu
@pytest.mark.parametrize("max_replica", [2, 3, 5])
def test_ring_locations_into_page_locked_host_memory(gpu, max_replica):
    """locs / counts in page-locked host memory (krk_host_alloc): the gather writes the owner
    lists there over PCIe -- the same lists as device outputs, word-aligned or not, u8 and
    int32; pageable host memory is refused (KRK_EINVAL) before any launch."""
    import ctypes as C
    labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(16)]
    healthy = np.ones(16, dtype=np.uint8)
    healthy[[4, 11]] = 0
    rng = np.random.default_rng(500 + max_replica)
    n = 20003
    digests = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    dbuf = D.DeviceBuffer(n * 32)
    dbuf.from_host(digests.reshape(-1))
    l8, c8 = D.DeviceBuffer(n * max_replica), D.DeviceBuffer(n)
    l32, c32 = D.DeviceBuffer(n * max_replica * 4), D.DeviceBuffer(n)
    D.ring_locations_u8_dev(dbuf, n, labels, healthy, max_replica, l8, c8)
    D.ring_locations_dev(dbuf, n, labels, healthy, max_replica, l32, c32)
    D.synchronize()
    w8, wc = l8.to_host(np.uint8, n * max_replica), c8.to_host(np.uint8, n)
    w32 = l32.to_host(np.int32, n * max_replica)
    pl, pc = D.PinnedArray((n * max_replica + 8,), np.uint8), D.PinnedArray((n + 8,), np.uint8)
    s, keep = D.nodes_struct(labels, [100] * 16)
    hp = healthy.ctypes.data_as(C.POINTER(C.c_uint8))
    for shift in (0, 1, 4):
        pl.a[:] = 0xAA
        pc.a[:] = 0xAA
        check(lib.krk_ring_locations_u8_dev(dbuf.ptr, n, C.byref(s), hp, max_replica, pl.ptr + shift, pc.ptr + shift,
                                             None))
        D.synchronize()
        assert np.array_equal(pl.a[shift:shift + n * max_replica], w8), shift
        assert np.array_equal(pc.a[shift:shift + n], wc), shift
        assert (pl.a[:shift] == 0xAA).all() and (pl.a[shift + n * max_replica:] == 0xAA).all()
    p32 = D.PinnedArray((n * max_replica,), np.int32)
    pc.a[:] = 0
    check(lib.krk_ring_locations_dev(dbuf.ptr, n, C.byref(s), hp, max_replica, p32.ptr, pc.ptr, None))
    D.synchronize()
    assert np.array_equal(p32.a, w32) and np.array_equal(pc.a[:n], wc)
    pageable = np.zeros(n * max_replica, dtype=np.uint8)
    with pytest.raises(Exception, match="page-locked"):
        check(lib.krk_ring_locations_u8_dev(dbuf.ptr, n, C.byref(s), hp, max_replica,
                                             pageable.ctypes.data, c8.ptr, None))
    D.synchronize()


@pytest.mark.parametrize("n_nodes", [3, 5, 16, 64])
def test_owner_table_every_row_matches_oracle(gpu, orc, n_nodes):
    """the WHOLE C5 output space.  With equal weights Locations depends
    on the digest only through its 2-byte ShardID (lib/hashring/ring.go:96-118 over
    lib/hrw/rendezvous.go:207-217), so the 65,536-row owner table is every result a ring can
    give.  For MaxReplica in {2, 3} and healthy in {all, a seeded 75 %, none}: every row of
    the device table (krk_ring_owner_table) equals the oracle's (orc_ring_owner_table) --
    owners, -1 padding and counts -- and 1M random digests gathered on the device (int32 and
    u8 / packed-row paths) equal the oracle table's row of their ShardID.  No row is sampled."""
    labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(n_nodes)]
    rng = np.random.default_rng(0xC5 + n_nodes)
    n = 1 << 20
    digests = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    shard = (digests[:, 0].astype(np.int64) << 8) | digests[:, 1]
    dbuf = D.DeviceBuffer(n * 32)
    dbuf.from_host(digests.reshape(-1))
    h75 = (rng.random(n_nodes) < 0.75).astype(np.uint8)
    h75[rng.integers(0, n_nodes)] = 1
    for max_replica in (2, 3):
        for healthy in (np.ones(n_nodes, np.uint8), h75, np.zeros(n_nodes, np.uint8)):
            want_l, want_c = orc.ring_owner_table(labels, [100] * n_nodes, healthy, max_replica)
            ring = hashring.Ring(labels, [l for l, h in zip(labels, healthy) if h], max_replica)
            ring.Refresh()
            got_l, got_c = ring._table
            bad = np.nonzero((got_l != want_l).any(axis=1) | (got_c != want_c))[0]
            assert bad.size == 0, (max_replica, healthy.tolist(), bad[:8], got_l[bad[:4]], want_l[bad[:4]])
            if not healthy.any() or healthy.all() and max_replica == 3:
                continue  # the gather legs below: one healthy set per replica count is enough
            l32, c32 = D.DeviceBuffer(n * max_replica * 4), D.DeviceBuffer(n)
            l8, c8 = D.DeviceBuffer(n * max_replica), D.DeviceBuffer(n)
            D.ring_locations_dev(dbuf, n, labels, healthy, max_replica, l32, c32)
            D.ring_locations_u8_dev(dbuf, n, labels, healthy, max_replica, l8, c8)
            D.synchronize()
            a32 = l32.to_host(np.int32, n * max_replica).reshape(n, max_replica)
            assert np.array_equal(a32, want_l[shard]), (max_replica, healthy.tolist())
            assert np.array_equal(c32.to_host(np.uint8, n), want_c[shard])
            a8 = l8.to_host(np.uint8, n * max_replica).reshape(n, max_replica)
            assert np.array_equal(a8, np.where(want_l < 0, 255, want_l).astype(np.uint8)[shard])
            assert np.array_equal(c8.to_host(np.uint8, n), want_c[shard])


def test_ring_locations_into_managed_memory(gpu):
    """outputs in managed memory (hipMallocManaged) are device-writable -- the
    placement kernels write them like device memory -- and give the device outputs' lists."""
    import ctypes as C
    hip = C.CDLL(D.lib._name)  # the HIP runtime the library itself links (not another copy in the process)
    hip.hipMallocManaged.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipFree.argtypes = [C.c_void_p]
    labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(16)]
    healthy = np.ones(16, dtype=np.uint8)
    n, R = 10007, 3
    rng = np.random.default_rng(42)
    digests = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    dbuf = D.DeviceBuffer(n * 32)
    dbuf.from_host(digests.reshape(-1))
    l8, c8 = D.DeviceBuffer(n * R), D.DeviceBuffer(n)
    D.ring_locations_u8_dev(dbuf, n, labels, healthy, R, l8, c8)
    D.synchronize()
    ml, mc = C.c_void_p(), C.c_void_p()
    assert hip.hipMallocManaged(C.byref(ml), n * R, 1) == 0 and hip.hipMallocManaged(C.byref(mc), n, 1) == 0
    try:
        s, keep = D.nodes_struct(labels, [100] * 16)
        check(lib.krk_ring_locations_u8_dev(dbuf.ptr, n, C.byref(s), healthy.ctypes.data_as(C.POINTER(C.c_uint8)), R,
                                             ml.value, mc.value, None))
        D.synchronize()
        got_l = np.ctypeslib.as_array((C.c_uint8 * (n * R)).from_address(ml.value)).copy()
        got_c = np.ctypeslib.as_array((C.c_uint8 * n).from_address(mc.value)).copy()
        assert np.array_equal(got_l, l8.to_host(np.uint8, n * R)) and np.array_equal(got_c, c8.to_host(np.uint8, n))
    finally:
        hip.hipFree(ml)
        hip.hipFree(mc)
