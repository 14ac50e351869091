#!/usr/bin/env python3
"""Instruction count of the production SHA-256 consumer loop, from the disassembly
of the gfx950 code object inside libkraken_hip.so (the ISA side of the per-stream
issue ceiling that bench.py reports for sha256_multi).

The .hip_fatbin section holds one clang offload bundle per translation unit; the one
with sha256_ws_kernel is unbundled and disassembled with the ROCm LLVM tools.  In the
two-lane kernel (sha256_ws_kernel<0, true, 1>) every instruction-round has exactly one
`v_add_u32_dpp ... row_mirror`, so the consumer's block loop is the backward-branch
loop whose body holds those DPP adds (one loop iteration = one producer step = two
blocks).  Per block we count every VALU instruction (the wave must issue each at >= 4
cycles when alone on its SIMD, MI355X_MICROARCH.md 'vector-instruction ISSUE cost'),
the 9-instruction rounds among them, and the LDS / SALU instructions beside them.

    python tools/sha_isa.py [lib.so] [--json out.json]
"""
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
KERNEL = "sha256_ws_kernel<0, true, 1>"  # two lanes per stream
KERNELS = {2: KERNEL, 8: "sha256_w8_kernel<0, 1>"}
# the one cross-lane add of every instruction-round, and the VALU ops of a round
ROUND_MARK = {2: "bitop3:0x96", 8: "quad_perm:[1,2,0,3]"}  # once per instruction-round
SELECT_MARK = {2: "row_mirror", 8: "quad_perm:[1,2,0,3]"}  # only in consumer code (finds its loop)
ROUND_OPS = {2: 9, 8: 8}
ROUNDS_PER_BLOCK = {2: 64, 8: 64}  # both consumers pipeline blocks (block2p, block8p)
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _disasm(lib_path: str, kernel: str = KERNEL) -> str:
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib_path, os.devnull],
                       check=True, capture_output=True)
        blob = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
        for k, a in enumerate(starts):
            e = starts[k + 1] if k + 1 < len(starts) else len(blob)
            b, o = os.path.join(td, f"b{k}.bin"), os.path.join(td, f"c{k}.o")
            open(b, "wb").write(blob[a:e])
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={b}", f"--output={o}"],
                               capture_output=True)
            if r.returncode:
                continue
            s = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--demangle", o], check=True, capture_output=True,
                               text=True).stdout
            if kernel in s:
                return s
    raise RuntimeError(f"{kernel} not found in {lib_path}")


def count(lib_path: str, lanes: int = 2) -> dict:
    kernel, mark, sel = KERNELS[lanes], ROUND_MARK[lanes], SELECT_MARK[lanes]
    lines = _disasm(lib_path, kernel).splitlines()
    head = [i for i, l in enumerate(lines) if l.endswith(">:") and kernel in l][0]
    nxt = [i for i, l in enumerate(lines) if i > head and l.endswith(">:")]
    body = lines[head + 1:nxt[0] if nxt else len(lines)]
    ins = []  # (address, text, branch target or None)
    for l in body:
        m = re.match(r"\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):\s*([0-9A-F]{8})(?: ([0-9A-F]{8}))?", l)
        if not m:
            continue
        t = re.search(r"\+0x([0-9a-f]+)>\s*$", l)
        ins.append((int(m.group(2), 16), m.group(1), t.group(1) if t else None, 4 if m.group(4) is None else 8))
    base = ins[0][0]
    loops = []
    for k, (a, t, tgt, _) in enumerate(ins):
        if tgt is not None and t.startswith(("s_cbranch", "s_branch")):
            dst = base + int(tgt, 16)  # objdump prints targets relative to the symbol start
            if dst <= a:
                loop = [x for x in ins if dst <= x[0] <= a]
                loops.append(loop)
    # the consumer's step loop: the shortest loop holding the most rounds (an inner
    # back-edge that re-runs only part of a step does not count as the step)
    most = max(sum(sel in x[1] for x in lp) for lp in loops)
    loop = min((lp for lp in loops if sum(sel in x[1] for x in lp) == most), key=len)
    dpp = sum(mark in x[1] for x in loop)
    blocks = dpp // ROUNDS_PER_BLOCK[lanes]
    assert blocks >= 1 and dpp == ROUNDS_PER_BLOCK[lanes] * blocks, dpp
    valu = sum(x[1].startswith("v_") for x in loop)
    lds = sum(x[1].startswith("ds_") for x in loop)
    salu = sum(x[1].startswith("s_") for x in loop)
    nbytes = sum(x[3] for x in loop)
    mix = {}
    for x in loop:
        op = x[1].split()[0]
        mix[op] = mix.get(op, 0) + 1
    return {"instruction_mix_per_iteration": dict(sorted(mix.items(), key=lambda kv: -kv[1])),"kernel": kernel, "lanes_per_stream": lanes, "loop_instructions": len(loop), "blocks_per_iteration": blocks,
            "instruction_rounds_per_block": dpp // blocks, "round_valu_per_block": ROUND_OPS[lanes] * (dpp // blocks),
            "valu_per_block": valu / blocks, "lds_per_block": lds / blocks, "salu_per_block": salu / blocks,
            "code_bytes_per_block": nbytes / blocks,
            "issue_cycles_per_valu": 4, "source": "llvm-objdump of the gfx950 code object in " +
            os.path.relpath(lib_path, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))}


def ceiling_mbps(isa: dict, clock_mhz: float) -> float:
    """Per-stream ceiling: one 64-byte block per (VALU per block x 4 cycles)."""
    return 64.0 * clock_mhz / (isa["valu_per_block"] * isa["issue_cycles_per_valu"])


# A lone wave's instruction stream, measured (tools/micro/vopcost.hip,
# profiles/r02/micro_vop_encoding_cost.txt): 8-byte encodings -- VOP3, DPP, and even a
# VOP2 or VOP1 carrying a 32-bit literal -- issue every 4.64 cycles, 4-byte VOP2 every
# 4.16, whatever the operands: the wave is fed about 8 B of code per 4.64 cycles.
FETCH_BYTES_PER_CYCLE = 8 / 4.64


def fetch_ceiling_mbps(isa: dict, clock_mhz: float) -> float:
    """Per-stream ceiling set by the consumer loop's code bytes at the measured fetch rate."""
    return 64.0 * clock_mhz / (isa["code_bytes_per_block"] / FETCH_BYTES_PER_CYCLE)


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    argv = sys.argv[1:]
    lanes = int(argv[argv.index("--lanes") + 1]) if "--lanes" in argv else 2
    args = [a for i, a in enumerate(argv) if not a.startswith("--") and (i == 0 or argv[i - 1] not in ("--lanes", "--json"))]
    lib = args[0] if args else os.path.join(root, "kraken_amd", "lib", "libkraken_hip.so")
    res = count(lib, lanes)
    res["ceiling_per_stream_MBps_at_2400MHz"] = round(ceiling_mbps(res, 2400.0), 3)
    res["fetch_ceiling_per_stream_MBps_at_2400MHz"] = round(fetch_ceiling_mbps(res, 2400.0), 3)
    print(json.dumps(res, indent=1))
    if "--json" in sys.argv:
        out = sys.argv[sys.argv.index("--json") + 1]
        json.dump(res, open(out, "w"), indent=1)
