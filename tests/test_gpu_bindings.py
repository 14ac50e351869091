"""The C side of INTEGRATION.md's cgo bindings, compiled (C11, -Wall -Werror) and run:
tests/native/bindings.c makes the calls the Go files make, with their argument shapes --
krk_init over every GPU with the defaults, NewMetaInfo's piece stream in 4 MiB reads with the
two-phase end, PieceHash writes that surface a failure, verifyPieces over pinned receive
buffers, verifyAndGenerate / pieceSumsFiles from files, an AUTO Digester that keeps writing
after Digest(), the ring's owner table -- and checks each against the host primitives."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu


def test_cgo_binding_shapes(gpu, tmp_path):
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "bindings")
    assert os.path.exists(exe), "build() compiles tests/native"
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"bindings_ok": True, "failures": 0}
