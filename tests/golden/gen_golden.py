"""Generates tests/golden/golden.json -- the fixtures that pin the CPU oracle.

Every expected value here is produced WITHOUT the oracle, by independent means:
Python's zlib.crc32 (= Go hash/crc32 IEEE), hashlib sha256/sha1 (= Go
crypto/sha256, crypto/sha1), and small pure-Python restatements of murmur3
x64_128 (spaolacci/murmur3 New64, glide.lock:231-232), Go math.Log
(src/math/log.go) and the bencode layout of core.info (core/metainfo.go:29-44).
Alongside them sit the reference's own known-answer tests, copied as data:
InfoHash KAT (core/metainfo_test.go:61-76), sha256("test")
(core/digester_test.go:27-28), DigestEmptyTar (core/digest.go:28), the
GetPieceLength table (core/metainfo_test.go:25-46), the piece-length ranges
(lib/metainfogen/config_test.go:23-38), and the published murmur3 test vectors.

Synthetic content follows the spec shared with oracle/oracle.c and
kraken_amd/csrc/synth_fill.hip, re-implemented here in numpy.

Run:  python tests/golden/gen_golden.py   (writes golden.json next to this file)
"""
import hashlib
import json
import math
import os
import struct
import zlib

import numpy as np

M64 = (1 << 64) - 1
GAMMA = 0x9E3779B97F4A7C15
ALNUM = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789"


# ------------------------------------------------------------- synthetic content

def _mix_np(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _mix(z):
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def synth(blob_idx: int, length: int, variant: int = 0) -> bytes:
    seed = _mix(((0x4B52414B454E ^ blob_idx) + GAMMA) & M64)
    nw = (length + 7) // 8
    with np.errstate(over="ignore"):
        j = np.arange(1, nw + 1, dtype=np.uint64)
        w = _mix_np(np.uint64(seed) + j * np.uint64(GAMMA))
    b = w.astype("<u8").tobytes()[:length]
    if variant:
        b = bytes(ALNUM[x % 62] for x in b)
    return b


# ------------------------------------------------------------- pieces

def piece_sums(data: bytes, P: int):
    out, off = [], 0
    while True:  # core/metainfo.go:162-177
        n = min(P, len(data) - off)
        if n == 0:
            break
        out.append(zlib.crc32(data[off:off + n]))
        off += n
        if n < P:
            break
    return out


def bencode_info(P, sums, name, length) -> bytes:
    s = b"d6:Lengthi%de4:Name%d:%s11:PieceLengthi%de9:PieceSumsl" % (length, len(name), name.encode(), P)
    s += b"".join(b"i%de" % x for x in sums)
    return s + b"ee"


# ------------------------------------------------------------- murmur3 / HRW

def _rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def _fmix(k):
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & M64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & M64
    return k ^ (k >> 33)


def murmur3_h1(data: bytes, seed: int = 0) -> int:
    c1, c2 = 0x87C37B91114253D5, 0x4CF5AD432745937F
    h1 = h2 = seed
    n = len(data)
    nb = n // 16
    for i in range(nb):
        k1, k2 = struct.unpack_from("<QQ", data, 16 * i)
        k1 = (_rotl((k1 * c1) & M64, 31) * c2) & M64
        h1 ^= k1
        h1 = (_rotl(h1, 27) + h2) & M64
        h1 = (h1 * 5 + 0x52DCE729) & M64
        k2 = (_rotl((k2 * c2) & M64, 33) * c1) & M64
        h2 ^= k2
        h2 = (_rotl(h2, 31) + h1) & M64
        h2 = (h2 * 5 + 0x38495AB5) & M64
    tail = data[16 * nb:]
    k1 = k2 = 0
    for i in range(len(tail) - 1, 7, -1):
        k2 = (k2 << 8) | tail[i]
    for i in range(min(len(tail), 8) - 1, -1, -1):
        k1 = (k1 << 8) | tail[i]
    if len(tail) > 8:
        h2 ^= (_rotl((k2 * c2) & M64, 33) * c1) & M64
    if len(tail) > 0:
        h1 ^= (_rotl((k1 * c1) & M64, 31) * c2) & M64
    h1 ^= n
    h2 ^= n
    h1 = (h1 + h2) & M64
    h2 = (h2 + h1) & M64
    h1, h2 = _fmix(h1), _fmix(h2)
    return (h1 + h2) & M64


def go_log(x: float) -> float:
    """src/math/log.go, op for op (Python floats are IEEE binary64, no fusing)."""
    Ln2Hi, Ln2Lo = 6.93147180369123816490e-01, 1.90821492927058770002e-10
    L1, L2, L3 = 6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01
    L4, L5, L6, L7 = 2.222219843214978396e-01, 1.818357216161805012e-01, 1.531383769920937332e-01, \
        1.479819860511658591e-01
    if math.isnan(x) or x == math.inf:
        return x
    if x < 0:
        return math.nan
    if x == 0:
        return -math.inf
    f1, ki = math.frexp(x)
    if f1 < math.sqrt(2) / 2:
        f1 *= 2
        ki -= 1
    f = f1 - 1
    k = float(ki)
    s = f / (2 + f)
    s2 = s * s
    s4 = s2 * s2
    t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)))
    t2 = s4 * (L2 + s4 * (L4 + s4 * L6))
    R = t1 + t2
    hfsq = 0.5 * f * f
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f)


def hrw_score(key_hex: str, label: str, weight: int) -> float:
    kb = bytes.fromhex(key_hex)
    h1 = murmur3_h1(kb + label.encode())
    val = h1 & ((1 << 53) - 1)
    if val == 0:  # rendezvous.go:111-116
        val = murmur3_h1(h1.to_bytes(8, "big")) & ((1 << 53) - 1)
    return -float(weight) / go_log(val / float(1 << 53))


def hrw_order(key_hex, labels, weights):
    sc = [hrw_score(key_hex, l, w) for l, w in zip(labels, weights)]
    order = sorted(range(len(labels)), key=lambda j: (-sc[j], j))
    return order, sc


def locations(order, healthy, max_replica):
    if not any(healthy):
        return [order[0]]
    out = []
    i = 0
    while i < len(order) and (not out or i < max_replica):
        if healthy[order[i]]:
            out.append(order[i])
        i += 1
    return out


def f64bits(x: float) -> str:
    return struct.pack(">d", x).hex()


# ------------------------------------------------------------- build

def main():
    rng = np.random.default_rng(20190402)
    g = {"about": __doc__.splitlines()[0]}
    g["kat"] = {
        "info_hash": {"piece_length": 4194304, "piece_sums": [2131691452],
                      "name": "289314c356bc2a19802c3e31505506db30ea81a0bcaea4ec3e079524c8ac3cf5",
                      "length": 236, "expected": "85b978c4377625b3963df406d0dd3a1da5a7d9c3"},
        "sha256_test": {"input": "test",
                        "expected": "9f86d081884c7d659a2feaa0c55ad015a3bf4f1b2b0b822cd15d6c15b0f00a08"},
        "digest_empty_tar": "sha256:e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
        "crc32_check": {"input": "123456789", "expected": 0xCBF43926},
        "get_piece_length": [[10, 3, 0, 3], [10, 3, 3, 1], [8, 2, 3, 2], [10, 3, 1, 3], [10, 3, 4, 0],
                             [10, 3, -1, 0]],
        "piece_length_ranges": {"ranges": [[0, 1 << 20], [2 << 30, 4 << 20], [4 << 30, 8 << 20]],
                                "cases": [[1 << 30, 1 << 20], [2 << 30, 4 << 20], [3 << 30, 4 << 20],
                                          [4 << 30, 8 << 20], [8 << 30, 8 << 20]]},
        "murmur3_h1": [["", "0000000000000000"], ["hello", "cbd8a7b341bd9b02"],
                       ["hello, world", "342fac623a5ebc8e"], ["19 Jan 2038 at 3:14:07 AM", "b89e5988b737affc"],
                       ["The quick brown fox jumps over the lazy dog.", "cd99481f9ee902c9"]],
        "rehash_inputs": [str(1 << (53 + i)) for i in range(11)],
    }
    # pieces: edge lengths x piece lengths, two content variants
    pieces = []
    lens = [0, 1, 2, 3, 7, 8, 10, 15, 16, 17, 63, 64, 65, 255, 256, 4095, 4096, 4097, 65536 + 7, 262145]
    for P in [1, 2, 3, 8, 10, 4096, 65536, 262144]:
        for L in lens:
            if L // P > 300:
                continue
            for variant in (0, 1):
                idx = 1000 * P + L
                data = synth(idx, L, variant)
                sums = piece_sums(data, P)
                pieces.append({"blob": idx, "variant": variant, "length": L, "piece_length": P,
                               "n": len(sums), "sums": sums,
                               "sha256": hashlib.sha256(data).hexdigest(),
                               "info_hash": hashlib.sha1(bencode_info(P, sums, hashlib.sha256(data).hexdigest(),
                                                                      L)).hexdigest()})
    g["pieces"] = pieces
    # a few larger blobs: only aggregate checks
    big = []
    for L, P in [(1 << 22, 1 << 20), ((1 << 22) + 12345, 1 << 20), (3 << 20, 262144)]:
        data = synth(L, L)
        sums = piece_sums(data, P)
        big.append({"blob": L, "length": L, "piece_length": P, "n": len(sums),
                    "sums_sha256": hashlib.sha256(np.asarray(sums, dtype="<u4").tobytes()).hexdigest(),
                    "sha256": hashlib.sha256(data).hexdigest()})
    g["big"] = big
    # HRW orders and score bits
    hrw = []
    for N, weighted in [(3, False), (5, False), (16, False), (64, False), (4, True), (16, True)]:
        labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(N)]
        weights = [[100, 200, 400, 800][i % 4] if weighted else 100 for i in range(N)]
        for nb in (1, 2, 32):
            for _ in range(12):
                key = rng.bytes(nb).hex()
                order, sc = hrw_order(key, labels, weights)
                hrw.append({"key": key, "labels": labels, "weights": weights, "order": order,
                            "score_bits": [f64bits(x) for x in sc]})
    g["hrw"] = hrw
    # ring.Locations
    ring = []
    for N, MR in [(3, 3), (5, 2), (16, 3), (4, 0)]:
        labels = [f"origin-{i:03d}.kraken.test:15002" for i in range(N)]
        for hp in (1.0, 0.6, 0.0):
            healthy = [1 if rng.random() < hp else 0 for _ in range(N)]
            for _ in range(10):
                d = rng.bytes(32)
                order, _ = hrw_order(d[:2].hex(), labels, [100] * N)
                ring.append({"digest": d.hex(), "labels": labels, "healthy": healthy, "max_replica": MR,
                             "locations": locations(order, healthy, MR)})
    g["ring"] = ring
    g["go_log"] = [[f64bits(x), f64bits(go_log(x))] for x in
                   [2.0 ** -53, 1e-10, 0.1, 0.25, 0.5, 0.7071067811865476, 0.75, 0.9, 0.999999, 1.0, 3.0]]
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")
    with open(out, "w") as f:
        json.dump(g, f, separators=(",", ":"))
    print(f"wrote {out}: {len(pieces)} piece cases, {len(hrw)} hrw cases, {len(ring)} ring cases")


if __name__ == "__main__":
    main()
