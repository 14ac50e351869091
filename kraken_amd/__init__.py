"""kraken_amd: MI355X-native blob-metainfo hot path (piece CRC-32, SHA-256
digests, HRW placement) behind a C ABI (include/kraken_hip.h).

Submodules mirror the reference packages they replace: ``core`` (core/),
``hrw`` (lib/hrw), ``hashring`` (lib/hashring Locations), ``metainfogen``
(lib/metainfogen).  ``device`` holds the device-resident batch helpers used by
bench.py.
"""
from ._capi import KrakenError, LIB_PATH, lib  # noqa: F401  (fails loudly if the HIP lib is missing)

__version__ = "0.1.0"
