#!/usr/bin/env python3
"""Lane-level model of the eight-lane SHA-256 consumer (sha256_multi.hip block8p):
one E lane and one A lane of a stream executing the same instruction stream with
per-lane operands, DPP cross reads seeing the partner's value from before the
instruction.  The quad-rotated Sigma is exact, so one lane per half suffices.
Checks the pipelined schedule (64 instruction-rounds a block, feed-forward and
compensation ops F1/F2/F3) against hashlib-equivalent compression on random blocks.
Development tool: run `python tools/sha8p_model.py`.
"""
import random
import struct

M = 0xFFFFFFFF
K = [0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
     0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
     0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
     0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
     0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
     0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
     0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
     0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2]
IV = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]


def rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M


def schedule(block):
    w = list(struct.unpack(">16I", block))
    for i in range(16, 64):
        s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3)
        s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10)
        w.append((w[i - 16] + s0 + w[i - 7] + s1) & M)
    return [(w[i] + K[i]) & M for i in range(64)]


def compress(h, kw):
    a, b, c, d, e, f, g, hh = h
    for r in range(64):
        t1 = (hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g & M)) + kw[r]) & M
        t2 = ((rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c))) & M
        hh, g, f, e, d, c, b, a = g, f, e, (d + t1) & M, c, b, a, (t1 + t2) & M
    return [(x + y) & M for x, y in zip(h, [a, b, c, d, e, f, g, hh])]


class Lane:
    def __init__(self, is_e):
        self.is_e = is_e
        self.mA = 0 if is_e else M
        self.r = {}


def sigma(lane, x):
    return (rotr(x, 6) ^ rotr(x, 11) ^ rotr(x, 25)) if lane.is_e else (rotr(x, 2) ^ rotr(x, 13) ^ rotr(x, 22))


def step(lanes, fn):
    """One instruction on both lanes: fn(lane, partner_old_regs) -> dict of writes."""
    old = [dict(l.r) for l in lanes]
    writes = [fn(l, old[1 - i]) for i, l in enumerate(lanes)]
    for l, w in zip(lanes, writes):
        l.r.update(w)


def round8(lanes, X0, X1, X2, NX, W):
    # alignbit/xor/xor -> t, k, F, P (cross add with the CURRENT z), z for the next round, add3
    def f(l, po):
        r = l.r
        t = sigma(l, r[X0])
        k = (r[X0] ^ (r[X1] & l.mA) ^ (~l.mA & M)) & M
        F = (k & r[X2]) | (~k & M & r[X1])
        P = (po[X1] + r["z"]) & M
        z = ((r[X2] ^ l.mA) + r[W]) & M
        return {"z": z, NX: (t + F + P) & M}
    step(lanes, f)


def run_stream(blocks_kw, H, nb_run):
    """E and A lane of one stream over blocks_kw (len = mine), nb_run >= mine blocks run."""
    E, A = Lane(True), Lane(False)
    lanes = [E, A]
    mine = len(blocks_kw)
    for l in lanes:
        h = H[4:8] if l.is_e else [H[k ^ 2] for k in range(4)]
        l.h = h
        l.r.update({"R0": h[0], "R3": h[1], "R2": h[2], "R1": h[3], "z": 0})
        l.r.update({f"hE{k}": (h[k] if l.is_e else 0) for k in range(4)})
        l.r.update({f"hA{k}": (0 if l.is_e else h[k]) for k in range(4)})
        l.mine = mine

    def W(l, i, r):  # W of block i, round r (A lanes: 1)
        if not l.is_e:
            return 1
        return blocks_kw[i][r] if i < mine else 0x12345678  # garbage past the stream

    def setW(i, r):
        for l in lanes:
            l.r["W"] = W(l, i, r)

    # prologue: z = xad(R1, mA, W0); round(R0,R3,R2,R1, W1); R1 <- h3 on A; round(R1,R0,R3,R2,W2); R2 <- h2 on A
    setW(0, 0)
    step(lanes, lambda l, po: {"z": ((l.r["R1"] ^ l.mA) + l.r["W"]) & M})
    setW(0, 1)
    round8(lanes, "R0", "R3", "R2", "R1", "W")
    A.r["R1"] = A.h[3]
    setW(0, 2)
    round8(lanes, "R1", "R0", "R3", "R2", "W")
    A.r["R2"] = A.h[2]
    for i in range(nb_run):
        # n = 2 .. 63: round n uses W of round n + 1 for z (n + 1 = 64 -> next block's W0)
        regs = ["R0", "R1", "R2", "R3"]
        for n in range(2, 64):
            X0, X1, X2, NX = regs[n % 4], regs[(n - 1) % 4], regs[(n - 2) % 4], regs[(n + 1) % 4]
            if n + 1 < 64:
                setW(i, n + 1)
            else:
                setW(i + 1, 0)
            round8(lanes, X0, X1, X2, NX, "W")
        # F1 (the kernel interleaves these with the R adds; the values are the same)
        step(lanes, lambda l, po: {"cc": (l.r["hA0"] - l.r["hE0"]) & M})
        step(lanes, lambda l, po: {"dd": (l.r["hA1"] - l.r["hE1"]) & M})
        step(lanes, lambda l, po: {"c2": po["cc"]})
        step(lanes, lambda l, po: {"z": (l.r["z"] + po["dd"]) & M})
        step(lanes, lambda l, po: {"z": (l.r["z"] + l.r["hE3"]) & M})
        for R, k in (("R0", 0), ("R3", 1), ("R2", 2), ("R1", 3)):
            step(lanes, lambda l, po, R=R, k=k: {R: (l.r[R] + l.r[f"hE{k}"]) & M})
        for R, k in (("R0", 0), ("R3", 1), ("R2", 2), ("R1", 3)):
            step(lanes, lambda l, po, R=R, k=k: {f"hE{k}": l.r[R] if i < (l.mine if l.is_e else 0) else l.r[f"hE{k}"]})
        setW(i + 1, 1)
        round8(lanes, "R0", "R3", "R2", "R1", "W")  # n = 64
        # F2
        step(lanes, lambda l, po: {"z": (l.r["z"] + l.r["c2"]) & M})
        setW(i + 1, 2)
        round8(lanes, "R1", "R0", "R3", "R2", "W")  # n = 65
        # F3
        step(lanes, lambda l, po: {"z": (l.r["z"] - l.r["hA1"]) & M})
        for R, k in (("R0", 0), ("R3", 1), ("R2", 2), ("R1", 3)):
            step(lanes, lambda l, po, R=R, k=k: {R: (l.r[R] + l.r[f"hA{k}"]) & M})
        for R, k in (("R0", 0), ("R3", 1), ("R2", 2), ("R1", 3)):
            step(lanes, lambda l, po, R=R, k=k: {f"hA{k}": l.r[R] if i < (0 if l.is_e else l.mine) else l.r[f"hA{k}"]})
    hE = [E.r[f"hE{k}"] for k in range(4)]
    hA = [A.r[f"hA{k}"] for k in range(4)]
    return [hA[2], hA[3], hA[0], hA[1]] + hE


if __name__ == "__main__":
    rnd = random.Random(7)
    bad = 0
    for trial in range(40):
        mine = rnd.randint(1, 5)
        extra = rnd.randint(0, 3)
        blocks = [bytes(rnd.getrandbits(8) for _ in range(64)) for _ in range(mine)]
        kws = [schedule(b) for b in blocks]
        H = IV if trial % 2 == 0 else [rnd.getrandbits(32) for _ in range(8)]
        ref = list(H)
        for kw in kws:
            ref = compress(ref, kw)
        got = run_stream(kws, H, mine + extra)
        if got != ref:
            bad += 1
            print("MISMATCH", trial, mine, extra, [hex(x) for x in got[:4]], [hex(x) for x in ref[:4]],
                  got[4:] == ref[4:])
    print("trials 40, bad", bad)
