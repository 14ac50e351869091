"""Host-side mirror of the reference's `core` package over the C ABI.

Names, argument meaning and error strings follow the Go API so callers (and the
parity tests) read like the reference:

* ``PieceHash``           core/piece_hash.go:21-24
* ``NewMetaInfo``         core/metainfo.go:53-79 (+ calcPieceSums :157-179)
* ``MetaInfo`` accessors  core/metainfo.go:81-155
* ``Digester``            core/digester.go:28-72
* ``Digest``              core/digest.go:51-161
* ``InfoHash``            core/infohash.go:25-60

All bulk arithmetic (piece CRCs, SHA-256) runs in libkraken_hip on the GPU; the
O(pieces) bencode + SHA-1 InfoHash runs in the same library's host code.
"""
from __future__ import annotations

import ctypes as C
import io
import json

import numpy as np

from ._capi import KrakenError, check, krk_blob, lib

SHA256 = "sha256"
DigestEmptyTar = "sha256:e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"
_COPY_BUF = 32 * 1024  # io.Copy's buffer: the Go reader granularity

_HEXB = frozenset(b"0123456789abcdefABCDEF")


def _go_quote(s: str) -> str:
    """fmt's %q for the common cases: double quotes, Go escapes."""
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch in '"\\':
            out.append("\\" + ch)
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\t":
            out.append("\\t")
        elif ch == "\r":
            out.append("\\r")
        elif ch.isprintable():
            out.append(ch)
        elif o < 0x80:
            out.append(f"\\x{o:02x}")
        elif o <= 0xFFFF:
            out.append(f"\\u{o:04x}")
        else:
            out.append(f"\\U{o:08x}")
    out.append('"')
    return "".join(out)


# ---------------------------------------------------------------- Digest

def ValidateSHA256(s: str) -> None:
    """core/digest.go:152-161: 64 BYTES (Go len) that hex.DecodeString accepts; the
    errors read like Go's ("hex: encoding/hex: invalid byte: U+0067 'g'")."""
    b = s.encode("utf-8", "surrogatepass")
    if len(b) != 64:
        raise ValueError(f"expected 64 characters, got {len(b)} from {_go_quote(s)}")
    for c in b:
        if c not in _HEXB:
            r = chr(c)
            shown = f" '{r}'" if r.isprintable() else ""
            raise ValueError(f"hex: encoding/hex: invalid byte: U+{c:04X}{shown}")


class Digest:
    __slots__ = ("_algo", "_hex", "_raw")

    def __init__(self, algo: str = "", hex_: str = "", raw: str = ""):
        self._algo, self._hex, self._raw = algo, hex_, raw

    def Algo(self) -> str:
        return self._algo

    def Hex(self) -> str:
        return self._hex

    def String(self) -> str:
        return self._raw

    __str__ = String

    def ShardID(self) -> str:
        """core/digest.go:148-150: the first 4 hex characters."""
        return self._hex[:4]

    def __eq__(self, other) -> bool:
        return isinstance(other, Digest) and (self._algo, self._hex, self._raw) == (
            other._algo, other._hex, other._raw)

    def __hash__(self) -> int:
        return hash(self._raw)

    def __repr__(self) -> str:
        return f"Digest({self._raw!r})"


def NewSHA256DigestFromHex(hex_: str) -> Digest:
    """core/digest.go:59-68."""
    try:
        ValidateSHA256(hex_)
    except ValueError as e:
        raise ValueError(f"invalid sha256: {e}") from None
    return Digest(SHA256, hex_, f"{SHA256}:{hex_}")


def ParseSHA256Digest(raw: str) -> Digest:
    """core/digest.go:72-93."""
    if raw == "":
        raise ValueError("invalid digest: empty")
    parts = raw.split(":")
    if len(parts) != 2:
        raise ValueError("invalid digest: expected '<algo>:<hex>'")
    if parts[0] != SHA256:
        raise ValueError("invalid digest algo: expected sha256")
    try:
        ValidateSHA256(parts[1])
    except ValueError as e:
        raise ValueError(f"invalid sha256: {e}") from None
    return Digest(parts[0], parts[1], raw)


class Digester:
    """core.Digester (core/digester.go:28-72).  Digest() does not reset, exactly like
    hash.Hash.Sum.  placement (krk_digester_new_on): PLACE_GPU batches this digester's
    bytes with every other GPU digester of the device into multi-stream SHA-256
    launches; PLACE_HOST runs SHA-NI on the calling thread; PLACE_AUTO (NewDigester)
    picks HOST while few digesters are live in the process, GPU beyond (the crossover
    in include/kraken_hip.h)."""

    def __init__(self, placement: int = 0):
        h = C.c_void_p()
        check(lib.krk_digester_new_on(placement, C.byref(h)))
        self._h = h

    def placement(self) -> int:
        v = C.c_int()
        check(lib.krk_digester_placement(self._h, C.byref(v)))
        return v.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.krk_digester_free(h)
            self._h = None

    def _write(self, p) -> int:
        b = _as_bytes(p)
        if b.nbytes:
            check(lib.krk_digester_write(self._h, b.ctypes.data, b.nbytes))
        return b.nbytes

    def Digest(self) -> Digest:
        out = (C.c_uint8 * 32)()
        check(lib.krk_digester_sum(self._h, out))
        return NewSHA256DigestFromHex(bytes(out).hex())

    def FromReader(self, rd) -> Digest:
        while True:
            chunk = rd.read(_COPY_BUF)
            if not chunk:
                break
            self._write(chunk)
        return self.Digest()

    def FromBytes(self, p) -> Digest:
        self._write(p)
        return self.Digest()

    def Tee(self, r):
        return _TeeReader(r, self)


PLACE_AUTO, PLACE_HOST, PLACE_GPU = 0, 1, 2


def NewDigester() -> Digester:
    return Digester(PLACE_AUTO)


class _TeeReader(io.RawIOBase):
    def __init__(self, r, d: Digester):
        self._r, self._d = r, d

    def readable(self):
        return True

    def read(self, n=-1):
        b = self._r.read(n)
        if b:
            self._d._write(b)
        return b

    def readinto(self, buf):
        b = self.read(len(buf))
        buf[: len(b)] = b
        return len(b)


# ---------------------------------------------------------------- InfoHash

class InfoHash(bytes):
    def Hex(self) -> str:
        return self.hex()

    def Bytes(self) -> bytes:
        return bytes(self)

    def String(self) -> str:
        return self.hex()


def NewInfoHashFromHex(s: str) -> InfoHash:
    """core/infohash.go:29-40."""
    if len(s) != 40:
        raise ValueError(f"invalid hash: expected 40 characters, got {len(s)}")
    try:
        return InfoHash(bytes.fromhex(s))
    except ValueError as e:
        raise ValueError(f"invalid hex: {e}") from None


def _info_hash(piece_length: int, sums: np.ndarray, name: str, length: int) -> InfoHash:
    s = np.ascontiguousarray(sums, dtype=np.uint32)
    out = (C.c_uint8 * 20)()
    nb = name.encode()
    sp = s.ctypes.data_as(C.POINTER(C.c_uint32)) if s.size else None
    check(lib.krk_info_hash(piece_length, sp, s.size, nb, len(nb), length, out))
    return InfoHash(bytes(out))


def _info_hash_batch(piece_lengths, sums: np.ndarray, sums_off, n_sums, names, lengths) -> list:
    """InfoHashes of many blobs in one call (krk_info_hash_batch, host threads):
    blob i's sums are sums[sums_off[i] : sums_off[i] + n_sums[i]]."""
    n = len(names)
    if not n:
        return []
    enc = [x.encode() for x in names]
    noff = np.zeros(n + 1, dtype=np.uint64)
    noff[1:] = np.cumsum([len(e) for e in enc])
    pl = np.ascontiguousarray(piece_lengths, dtype=np.int64)
    so = np.ascontiguousarray(sums_off, dtype=np.uint64)
    ns = np.ascontiguousarray(n_sums, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.int64)
    s = np.ascontiguousarray(sums, dtype=np.uint32)
    out = np.zeros(20 * n, dtype=np.uint8)
    check(lib.krk_info_hash_batch(pl.ctypes.data_as(C.POINTER(C.c_int64)),
                                  s.ctypes.data_as(C.POINTER(C.c_uint32)) if s.size else None,
                                  so.ctypes.data_as(C.POINTER(C.c_uint64)), ns.ctypes.data_as(C.POINTER(C.c_uint64)),
                                  b"".join(enc) or None, noff.ctypes.data_as(C.POINTER(C.c_uint64)),
                                  ln.ctypes.data_as(C.POINTER(C.c_int64)), n, out.ctypes.data_as(C.POINTER(C.c_uint8))))
    return [InfoHash(bytes(out[20 * i:20 * i + 20])) for i in range(n)]


# ---------------------------------------------------------------- MetaInfo

class MetaInfo:
    """core.MetaInfo (core/metainfo.go:46-155)."""

    def __init__(self, piece_length: int, piece_sums: np.ndarray | None, name: str, length: int,
                 digest: Digest, info_hash: InfoHash):
        self._pl = int(piece_length)
        self._sums = None if piece_sums is None else np.asarray(piece_sums, dtype=np.uint32)
        self._name = name
        self._len = int(length)
        self._digest = digest
        self._ih = info_hash

    def InfoHash(self) -> InfoHash:
        return self._ih

    def Digest(self) -> Digest:
        return self._digest

    def Length(self) -> int:
        return self._len

    def NumPieces(self) -> int:
        return 0 if self._sums is None else int(self._sums.size)

    def PieceLength(self) -> int:
        return self._pl

    def GetPieceLength(self, i: int) -> int:
        """core/metainfo.go:108-118."""
        n = self.NumPieces()
        if i < 0 or i >= n:
            return 0
        if i == n - 1:
            return self._len - self._pl * i
        return self._pl

    def GetPieceSum(self, i: int) -> int:
        return int(self._sums[i])

    def PieceSums(self) -> np.ndarray:
        return np.zeros(0, dtype=np.uint32) if self._sums is None else self._sums

    def Serialize(self) -> bytes:
        """core/metainfo.go:131-134: json of {"Info": info} (field order as declared)."""
        sums = None if self._sums is None else [int(x) for x in self._sums]
        obj = {"Info": {"PieceLength": self._pl, "PieceSums": sums, "Name": self._name,
                        "Length": self._len}}
        return json.dumps(obj, separators=(",", ":")).encode()


class _JObj(list):
    """A JSON object as its (key, value) pairs in document order (duplicates kept)."""


class _JNum(str):
    """A JSON number that is not an integer literal, kept as its text."""


def _go_kind(v) -> str:
    if isinstance(v, _JObj):
        return "object"
    if isinstance(v, list):
        return "array"
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, (int, _JNum)):
        return "number"
    return "string"


def _type_error(v, field: str, gotype: str) -> ValueError:
    what = f"number {v}" if isinstance(v, (int, _JNum)) and not isinstance(v, bool) else _go_kind(v)
    return ValueError(f"cannot unmarshal {what} into Go struct field {field} of type {gotype}")


_INFO_FIELDS = {"PieceLength": "int64", "PieceSums": "[]uint32", "Name": "string", "Length": "int64"}


def _match_field(key: str, fields) -> str | None:
    """encoding/json field lookup: the exact name, else a case-insensitive match."""
    if key in fields:
        return key
    return next((f for f in fields if f.lower() == key.lower()), None)


def _decode_info(pairs) -> dict:
    """json.Unmarshal of an object into core.info (core/metainfo.go:29-35): keys are
    applied in document order (a later duplicate wins); null leaves an int64 / string
    field unchanged and sets the slice to nil; a value of the wrong kind, or a number
    outside the field's range, is Go's UnmarshalTypeError."""
    out = {"PieceLength": 0, "PieceSums": None, "Name": "", "Length": 0}
    for key, v in pairs:
        f = _match_field(key, _INFO_FIELDS)
        if f is None:
            continue
        field = f"info.{f}"
        if f in ("PieceLength", "Length"):
            if v is None:
                continue
            if isinstance(v, bool) or not isinstance(v, int) or not -(1 << 63) <= v < (1 << 63):
                raise _type_error(v, field, "int64")
            out[f] = v
        elif f == "Name":
            if v is None:
                continue
            if not isinstance(v, str) or isinstance(v, _JNum):
                raise _type_error(v, field, "string")
            out[f] = str(v)
        else:
            if v is None:
                out[f] = None
                continue
            if not isinstance(v, list) or isinstance(v, _JObj):
                raise _type_error(v, field, "[]uint32")
            for x in v:
                if isinstance(x, bool) or not isinstance(x, int) or not 0 <= x < (1 << 32):
                    raise _type_error(x, field, "uint32")
            out[f] = list(v)
    return out


def DeserializeMetaInfo(data: bytes) -> MetaInfo:
    """core/metainfo.go:136-155 with encoding/json's rules for metaInfoJSON: missing
    fields and a null Info take Go's zero values, so a truncated sidecar fails the way
    the reference does ("parse name: invalid sha256: ..."); type and range errors read
    "json: cannot unmarshal <kind> into Go struct field info.<Field> of type <T>"."""
    try:
        j = json.loads(data, object_pairs_hook=_JObj, parse_float=_JNum)
        if j is None:
            j = _JObj()
        if not isinstance(j, _JObj):
            raise ValueError(f"cannot unmarshal {_go_kind(j)} into Go value of type core.metaInfoJSON")
        info = _JObj()
        for key, v in j:
            if _match_field(key, ("Info",)) is None or v is None:
                continue
            if not isinstance(v, _JObj):
                raise ValueError(f"cannot unmarshal {_go_kind(v)} into Go struct field metaInfoJSON.Info "
                                 "of type core.info")
            info = _JObj(list(info) + list(v))  # a repeated Info key merges into the same struct
        fields = _decode_info(info)
    except (ValueError, TypeError) as e:
        raise ValueError(f"json: {e}") from None
    pl, sums, name, length = fields["PieceLength"], fields["PieceSums"], fields["Name"], fields["Length"]
    arr = None if sums is None else np.asarray(sums, dtype=np.uint32)
    ih = _info_hash(pl, arr if arr is not None else np.zeros(0, np.uint32), name, length)
    try:
        d = NewSHA256DigestFromHex(name)
    except ValueError as e:
        raise ValueError(f"parse name: {e}") from None
    return MetaInfo(pl, arr, name, length, d, ih)


def _as_bytes(p) -> np.ndarray:
    if isinstance(p, np.ndarray):
        return np.ascontiguousarray(p).view(np.uint8).reshape(-1)
    return np.frombuffer(memoryview(p).cast("B"), dtype=np.uint8)


def _reader(blob):
    if isinstance(blob, (bytes, bytearray, memoryview, np.ndarray)):
        return io.BytesIO(_as_bytes(blob).tobytes())
    return blob


def calcPieceSums(blob, piece_length: int):
    """core.calcPieceSums (core/metainfo.go:157-179) on the GPU: the reader is
    copied through the C ABI's streaming piece API in io.Copy-sized chunks; CRC
    state crosses chunk and piece boundaries on the device."""
    if piece_length <= 0:
        raise ValueError("piece length must be positive")
    rd = _reader(blob)
    h = C.c_void_p()
    check(lib.krk_piece_stream_begin(piece_length, C.byref(h)))
    try:
        while True:
            try:
                chunk = rd.read(_COPY_BUF)
            except Exception as e:  # io error -> "read blob: %s"
                raise IOError(f"read blob: {e}") from None
            if not chunk:
                break
            b = _as_bytes(chunk)
            check(lib.krk_piece_stream_update(h, b.ctypes.data, b.nbytes))
        n = C.c_uint64()
        ln = C.c_uint64()
        check(lib.krk_piece_stream_end(h, None, 0, C.byref(n), C.byref(ln)))
        sums = np.zeros(max(n.value, 1), dtype=np.uint32)
        check(lib.krk_piece_stream_end(h, sums.ctypes.data_as(C.POINTER(C.c_uint32)), n.value,
                                       C.byref(n), C.byref(ln)))
        return ln.value, (sums[: n.value] if n.value else None)
    finally:
        lib.krk_piece_stream_free(h)


def NewMetaInfo(d: Digest, blob, piece_length: int) -> MetaInfo:
    """core.NewMetaInfo (core/metainfo.go:53-79).  Assumes d is the valid digest."""
    length, sums = calcPieceSums(blob, piece_length)
    ih = _info_hash(piece_length, sums if sums is not None else np.zeros(0, np.uint32), d.Hex(), length)
    return MetaInfo(piece_length, sums, d.Hex(), length, d, ih)


class _PieceHash32:
    """hash.Hash32 returned by PieceHash(): crc32.NewIEEE semantics; Sum32 runs the
    GPU kernel over the bytes written since the last Sum32 (state carried)."""

    def __init__(self):
        self._crc = 0
        self._pending: list[bytes] = []

    def Write(self, p) -> int:
        b = bytes(_as_bytes(p))
        self._pending.append(b)
        return len(b)

    def _fold(self):
        if self._pending:
            buf = np.frombuffer(b"".join(self._pending), dtype=np.uint8)
            self._pending = []
            out = C.c_uint32()
            check(lib.krk_crc32_update(self._crc, buf.ctypes.data if buf.size else None, buf.size,
                                       C.byref(out)))
            self._crc = out.value

    def Sum32(self) -> int:
        self._fold()
        return self._crc

    def Sum(self, b: bytes = b"") -> bytes:
        return bytes(b) + self.Sum32().to_bytes(4, "big")

    def Reset(self):
        self._crc, self._pending = 0, []

    def Size(self) -> int:
        return 4

    def BlockSize(self) -> int:
        return 1


def PieceHash() -> _PieceHash32:
    return _PieceHash32()


__all__ = ["Digest", "Digester", "NewDigester", "NewSHA256DigestFromHex", "ParseSHA256Digest",
           "ValidateSHA256", "InfoHash", "NewInfoHashFromHex", "MetaInfo", "NewMetaInfo",
           "DeserializeMetaInfo", "PieceHash", "calcPieceSums", "DigestEmptyTar", "KrakenError",
           "krk_blob"]
