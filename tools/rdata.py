"""Minimal reader for R's serialized `.rda` files (RDX2/RDX3, XDR binary).

Used only to turn the reference's example datasets (`data/es.mef.small.rda`,
`data/o.ifm.rda`, `data/knn.rda`) into small numpy fixtures under
`tests/golden/`.  It executes nothing from the file: it is a pure data parser
for the subset of the R serialization format those files use (pairlists,
symbols, atomic vectors, lists, attributes, references).

Format notes (R Internals, "Serialization Formats"):
  * the file is gzip/bzip2/xz compressed; payload starts with ``RDX2\n`` or
    ``RDX3\n`` followed by the format marker ``X\n`` (XDR, big-endian);
  * header: version, writer version, min reader version (+ native encoding
    for version 3);
  * each item starts with a 32-bit flags word: type = flags & 0xff,
    has-attr = bit 9, has-tag = bit 10.
"""
from __future__ import annotations

import bz2
import gzip
import lzma
import struct

import numpy as np

NILVALUE_SXP = 254
GLOBALENV_SXP = 253
UNBOUNDVALUE_SXP = 252
MISSINGARG_SXP = 251
BASENAMESPACE_SXP = 250
NAMESPACESXP = 249
PACKAGESXP = 248
PERSISTSXP = 247
EMPTYENV_SXP = 242
BASEENV_SXP = 241
ATTRLANGSXP = 240
ATTRLISTSXP = 239
ALTREP_SXP = 238
REFSXP = 255

NA_INTEGER = -(2 ** 31)


class RObject:
    """An R value: `.value` (numpy array / list / str / dict) and `.attrs`."""

    def __init__(self, rtype, value, attrs=None):
        self.rtype = rtype
        self.value = value
        self.attrs = attrs or {}

    def __repr__(self):  # pragma: no cover - debugging helper
        return f"RObject(type={self.rtype}, attrs={list(self.attrs)})"


def _decompress(raw: bytes) -> bytes:
    if raw[:2] == b"\x1f\x8b":
        return gzip.decompress(raw)
    if raw[:3] == b"BZh":
        return bz2.decompress(raw)
    if raw[:6] == b"\xfd7zXZ\x00":
        return lzma.decompress(raw)
    return raw


class _Reader:
    def __init__(self, buf: bytes):
        self.buf = buf
        self.pos = 0
        self.refs = []

    def int(self) -> int:
        v = struct.unpack_from(">i", self.buf, self.pos)[0]
        self.pos += 4
        return v

    def length(self) -> int:
        n = self.int()
        if n == -1:
            hi = self.int()
            lo = self.int()
            n = (hi << 32) + lo
        return n

    def bytes(self, n: int) -> bytes:
        b = self.buf[self.pos:self.pos + n]
        self.pos += n
        return b

    def item(self):
        flags = self.int()
        t = flags & 0xFF
        has_attr = bool(flags & (1 << 9))
        has_tag = bool(flags & (1 << 10))
        if t == NILVALUE_SXP:
            return None
        if t in (GLOBALENV_SXP, UNBOUNDVALUE_SXP, MISSINGARG_SXP,
                 BASENAMESPACE_SXP, EMPTYENV_SXP, BASEENV_SXP):
            return RObject(t, None)
        if t == REFSXP:
            idx = flags >> 8
            if idx == 0:
                idx = self.int()
            return self.refs[idx - 1]
        if t in (PERSISTSXP,):
            self.item()
            o = RObject(t, None)
            self.refs.append(o)
            return o
        if t in (NAMESPACESXP, PACKAGESXP):
            self.int()  # 0
            n = self.int()
            info = [self.item() for _ in range(n)]
            o = RObject(t, info)
            self.refs.append(o)
            return o
        if t == 1:  # SYMSXP
            name = self.item()
            o = RObject(1, name.value if isinstance(name, RObject) else name)
            self.refs.append(o)
            return o
        if t == 4:  # ENVSXP
            self.int()  # locked
            o = RObject(4, None)
            self.refs.append(o)
            enclos = self.item()
            frame = self.item()
            hashtab = self.item()
            attrib = self.item()
            o.value = {"enclos": enclos, "frame": frame, "hashtab": hashtab}
            o.attrs = attrib or {}
            return o
        if t in (2, 3, 5, 6, 17, ATTRLANGSXP, ATTRLISTSXP):  # pairlist-like
            attrs = self.item() if has_attr else None
            tag = self.item() if has_tag else None
            car = self.item()
            cdr = self.item()
            node = RObject(t, (tag, car, cdr))
            if attrs is not None:
                node.attrs = _pairlist_to_dict(attrs)
            return node
        if t == 9:  # CHARSXP
            n = self.int()
            if n == -1:
                return RObject(9, None)
            return RObject(9, self.bytes(n).decode("utf-8", "replace"))
        if t in (10, 13):  # LGLSXP, INTSXP
            n = self.length()
            v = np.frombuffer(self.bytes(4 * n), dtype=">i4").astype(np.int32)
            o = RObject(t, v)
        elif t == 14:  # REALSXP
            n = self.length()
            v = np.frombuffer(self.bytes(8 * n), dtype=">f8").astype(np.float64)
            o = RObject(t, v)
        elif t == 15:  # CPLXSXP
            n = self.length()
            v = np.frombuffer(self.bytes(16 * n), dtype=">f8").astype(np.float64)
            o = RObject(t, v[0::2] + 1j * v[1::2])
        elif t == 16:  # STRSXP
            n = self.length()
            o = RObject(t, [self.item().value for _ in range(n)])
        elif t in (19, 20):  # VECSXP, EXPRSXP
            n = self.length()
            o = RObject(t, [self.item() for _ in range(n)])
        elif t == 24:  # RAWSXP
            n = self.length()
            o = RObject(t, self.bytes(n))
        elif t == 25:  # S4SXP
            o = RObject(t, None)
        else:
            raise ValueError(f"unsupported SEXP type {t} at byte {self.pos}")
        if has_attr:
            o.attrs = _pairlist_to_dict(self.item())
        return o


def _pairlist_to_dict(node):
    out = {}
    while node is not None and isinstance(node, RObject) and node.rtype in (2, ATTRLISTSXP):
        tag, car, cdr = node.value
        key = tag.value if isinstance(tag, RObject) else str(len(out))
        out[key] = car
        node = cdr
    return out


def read_rda(path: str) -> dict:
    """Return {name: RObject} for every object saved in an .rda file."""
    with open(path, "rb") as f:
        raw = _decompress(f.read())
    if raw[:5] not in (b"RDX2\n", b"RDX3\n"):
        raise ValueError("not an RDX2/RDX3 file")
    r = _Reader(raw[5:])
    fmt = r.bytes(2)
    if fmt != b"X\n":
        raise ValueError("only XDR-format .rda files are supported")
    version = r.int()
    r.int()
    r.int()
    if version == 3:
        n = r.int()
        r.bytes(n)
    top = r.item()
    return _pairlist_to_dict(top)


def data_frame(obj: RObject):
    """Convert an R data.frame RObject to (column names, row names, {col: ndarray})."""
    names = obj.attrs["names"].value
    rn = obj.attrs.get("row.names")
    cols = {}
    for nm, col in zip(names, obj.value):
        cols[nm] = col.value
    nrow = len(obj.value[0].value) if obj.value else 0
    if rn is None:
        rownames = None
    elif rn.rtype == 16:
        rownames = list(rn.value)
    else:  # compact integer row names c(NA, -n)
        rownames = [str(i + 1) for i in range(nrow)]
    return list(names), rownames, cols
