"""the drop-in paths with the library's DEFAULTS -- run in a fresh
process with no knobs set (no krk_set_sha_host_offload, no placement, no KRK_ environment),
bit for bit against hashlib / zlib:

* a C1-shaped batch (one 1 GiB blob, 4 MiB pieces, core/metainfo.go:53-79 + the upload
  digest of origin/blobserver/uploader.go:74-94) through krk_metainfo_digest_dev: the
  planner hands the one long chain to a host thread (SHA-NI, read out of HBM) while the GPU
  computes the piece CRCs;
* one 1 GiB NewMetaInfo piece stream fed 4 MiB reads (core/metainfo.go:157-179): the AUTO
  crossover keeps a lone stream on its caller's thread.

This parity test asserts the outputs and the placements the defaults chose (the probe
script itself asserts them, bench.DEFAULTS_PROBE).  The rates -- the C1 call against one
host thread's SHA-NI time, the stream against one thread's PCLMUL rate -- are measured and
reported by `bench.py --workload defaults` (no -m gpu test asserts a
time)."""
import json
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_defaults_c1_and_piece_stream_outputs_and_placements(gpu):
    res = bench.run_defaults_probe(runs=1)
    print(res)
    assert res["stream_placement"] == "host" and res["digest_ok"] and res["sums_ok"]
