"""Universal Binary JSON codec in the dialect XGBoost 3.0 writes for models.

The shipped reference checkpoint (``src/api/models/xgb_model_tree.pkl``) wraps a
UBJSON document ``{"Config": ..., "Model": ...}``. XGBoost's dialect:

* object keys are written without the ``S`` marker: ``<int marker><length><utf-8 bytes>``;
* homogeneous numeric arrays are "optimised" containers ``[$<type>#<count marker><n>`` followed by
  ``n`` big-endian values (``d`` f32, ``l`` i32, ``U`` u8, ``L`` i64);
* all lengths and counts use the ``L`` (int64) marker.

Typed arrays decode to ``numpy`` arrays (native byte order); everything else to plain Python.
"""
from __future__ import annotations

import struct
from typing import Any

import numpy as np

_INT_FMT = {b"i": (">b", 1), b"U": (">B", 1), b"I": (">h", 2), b"l": (">i", 4), b"L": (">q", 8)}
_NUM_FMT = {**_INT_FMT, b"d": (">f", 4), b"D": (">d", 8)}
_NP_OF = {b"i": ">i1", b"U": ">u1", b"I": ">i2", b"l": ">i4", b"L": ">i8", b"d": ">f4", b"D": ">f8"}
_MARK_OF_NP = {np.dtype("int8"): b"i", np.dtype("uint8"): b"U", np.dtype("int16"): b"I",
               np.dtype("int32"): b"l", np.dtype("int64"): b"L", np.dtype("float32"): b"d",
               np.dtype("float64"): b"D"}


class UBJSONError(ValueError):
    pass


class _Reader:
    __slots__ = ("buf", "pos")

    def __init__(self, buf: bytes | bytearray | memoryview):
        self.buf = memoryview(buf)
        self.pos = 0

    def take(self, n: int) -> memoryview:
        if self.pos + n > len(self.buf):
            raise UBJSONError("truncated UBJSON document")
        v = self.buf[self.pos:self.pos + n]
        self.pos += n
        return v

    def marker(self) -> bytes:
        m = bytes(self.take(1))
        while m == b"N":  # no-op padding
            m = bytes(self.take(1))
        return m

    def number(self, m: bytes):
        fmt, size = _NUM_FMT[m]
        return struct.unpack(fmt, self.take(size))[0]

    def length(self) -> int:
        m = self.marker()
        if m not in _INT_FMT:
            raise UBJSONError(f"bad length marker {m!r}")
        n = self.number(m)
        if n < 0:
            raise UBJSONError("negative length")
        return n

    def string(self) -> str:
        return bytes(self.take(self.length())).decode("utf-8")

    def value(self, m: bytes | None = None) -> Any:
        if m is None:
            m = self.marker()
        if m in _NUM_FMT:
            return self.number(m)
        if m == b"S":
            return self.string()
        if m == b"C":
            return bytes(self.take(1)).decode("latin-1")
        if m == b"T":
            return True
        if m == b"F":
            return False
        if m == b"Z":
            return None
        if m == b"H":  # high-precision number as string
            s = self.string()
            return float(s) if any(c in s for c in ".eE") else int(s)
        if m == b"[":
            return self.array()
        if m == b"{":
            return self.obj()
        raise UBJSONError(f"unknown marker {m!r} at {self.pos - 1}")

    def _container_header(self):
        typ = cnt = None
        save = self.pos
        m = self.marker()
        if m == b"$":
            typ = self.marker()
            m = self.marker()
            if m != b"#":
                raise UBJSONError("typed container without count")
        if m == b"#":
            cnt = self.length()
        else:
            self.pos = save
        return typ, cnt

    def array(self):
        typ, cnt = self._container_header()
        if typ is not None:
            if typ in _NP_OF:
                dt = np.dtype(_NP_OF[typ])
                raw = self.take(cnt * dt.itemsize)
                return np.frombuffer(raw, dtype=dt).astype(dt.newbyteorder("="))
            return [self.value(typ) for _ in range(cnt)]
        if cnt is not None:
            return [self.value() for _ in range(cnt)]
        out = []
        while True:
            m = self.marker()
            if m == b"]":
                return out
            out.append(self.value(m))

    def obj(self):
        typ, cnt = self._container_header()
        out: dict[str, Any] = {}
        if cnt is not None:
            for _ in range(cnt):
                k = self.string()
                out[k] = self.value(typ) if typ is not None else self.value()
            return out
        while True:
            save = self.pos
            m = self.marker()
            if m == b"}":
                return out
            self.pos = save
            k = self.string()
            out[k] = self.value()


def loads(buf: bytes | bytearray | memoryview) -> Any:
    r = _Reader(buf)
    v = r.value()
    return v


# --------------------------------------------------------------------------------------- encoder

def _len(n: int) -> bytes:
    return b"L" + struct.pack(">q", n)


def _enc(v: Any, out: list[bytes]) -> None:
    if v is None:
        out.append(b"Z")
    elif v is True:
        out.append(b"T")
    elif v is False:
        out.append(b"F")
    elif isinstance(v, (int, np.integer)):
        i = int(v)
        # XGBoost picks the narrowest marker with a strict upper bound (127 -> 'I').
        if -128 <= i < 127:
            out.append(b"i" + struct.pack(">b", i))
        elif -32768 <= i < 32767:
            out.append(b"I" + struct.pack(">h", i))
        elif -2**31 <= i < 2**31 - 1:
            out.append(b"l" + struct.pack(">i", i))
        else:
            out.append(b"L" + struct.pack(">q", i))
    elif isinstance(v, (float, np.floating)):
        if isinstance(v, np.float32):
            out.append(b"d" + struct.pack(">f", float(v)))
        else:
            out.append(b"D" + struct.pack(">d", float(v)))
    elif isinstance(v, str):
        b = v.encode("utf-8")
        out.append(b"S" + _len(len(b)) + b)
    elif isinstance(v, np.ndarray):
        dt = v.dtype
        if dt == np.bool_:
            v = v.astype(np.uint8)
            dt = v.dtype
        if dt not in _MARK_OF_NP:
            raise UBJSONError(f"unsupported array dtype {dt}")
        m = _MARK_OF_NP[dt]
        out.append(b"[$" + m + b"#" + _len(v.size))
        out.append(np.ascontiguousarray(v, dtype=dt.newbyteorder(">")).tobytes())
    elif isinstance(v, dict):
        out.append(b"{")
        for k, x in v.items():
            kb = str(k).encode("utf-8")
            out.append(_len(len(kb)) + kb)
            _enc(x, out)
        out.append(b"}")
    elif isinstance(v, (list, tuple)):
        out.append(b"[#" + _len(len(v)))
        for x in v:
            _enc(x, out)
    else:
        raise UBJSONError(f"cannot encode {type(v).__name__}")


def dumps(v: Any) -> bytes:
    out: list[bytes] = []
    _enc(v, out)
    return b"".join(out)
