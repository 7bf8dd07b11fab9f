"""Static pickle codec for the XGBoost-compatible ``xgb_model_tree.pkl`` checkpoint.

The reference persists its model with ``joblib.dump(best_model_tree)``
(src/model_train_test/model_tree_train_test.py:215-219) and serves it with ``joblib.load``
(src/api/cobalt_fast_api.py:45). Unpickling executes arbitrary callables, so this module never
unpickles: :func:`decode` walks the opcode stream with :mod:`pickletools` and evaluates only data
opcodes (ints, floats, strings, bytes, tuples, lists, dicts). Global references and calls are kept
as inert :class:`GlobalRef` / :class:`Call` records, and only two known data patterns are lowered to
values: ``builtins.bytearray(bytes)`` and the numpy scalar ``numpy.core.multiarray.scalar(dtype, raw)``.

:func:`encode_xgb_classifier` writes the same opcode structure as joblib/pickle protocol 4 for an
``xgboost.sklearn.XGBClassifier`` (state dict + ``_Booster.handle`` = UBJSON bytearray), so a file
written here is loadable by real xgboost + joblib and by :func:`decode`.
"""
from __future__ import annotations

import io
import math
import pickletools
import struct
from dataclasses import dataclass, field
from typing import Any

import numpy as np


@dataclass(frozen=True)
class GlobalRef:
    module: str
    name: str

    @property
    def qualname(self) -> str:
        return f"{self.module}.{self.name}"


@dataclass
class Call:
    """An un-executed ``callable(*args)`` (REDUCE/NEWOBJ) plus the state a BUILD would apply."""

    func: GlobalRef
    args: tuple
    state: Any = None
    items: list = field(default_factory=list)


class _Mark:
    pass


_MARK = _Mark()


class PickleDecodeError(ValueError):
    pass


def _lower(obj: Any) -> Any:
    """Lower the few safe, known data patterns to Python/numpy values."""
    if isinstance(obj, Call):
        q = obj.func.qualname
        if q == "builtins.bytearray" and len(obj.args) == 1 and isinstance(obj.args[0], (bytes, bytearray)):
            return bytes(obj.args[0])
        if q in ("numpy.core.multiarray.scalar", "numpy._core.multiarray.scalar") and len(obj.args) == 2:
            dt, raw = obj.args
            if isinstance(dt, Call) and dt.func.name == "dtype" and isinstance(raw, (bytes, bytearray)):
                code = dt.args[0]
                endian = "<"
                if isinstance(dt.state, tuple) and len(dt.state) > 1 and dt.state[1] in ("<", ">", "|", "="):
                    endian = "<" if dt.state[1] in ("<", "|", "=") else ">"
                return np.frombuffer(bytes(raw), dtype=np.dtype(endian + code))[0]
    return obj


def decode(data: bytes) -> Any:
    """Statically decode a pickle byte string into data (never imports or calls anything)."""
    stack: list[Any] = []
    memo: dict[int, Any] = {}
    for op, arg, _pos in pickletools.genops(data):
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        if name == "STOP":
            break
        if name == "MARK":
            stack.append(_MARK)
        elif name in ("NONE",):
            stack.append(None)
        elif name in ("NEWTRUE", "NEWFALSE"):
            stack.append(name == "NEWTRUE")
        elif name in ("BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG"):
            stack.append(arg if not isinstance(arg, bool) else int(arg))
        elif name in ("BINFLOAT", "FLOAT"):
            stack.append(float(arg))
        elif name in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE", "SHORT_BINSTRING",
                      "BINSTRING", "STRING"):
            stack.append(arg if isinstance(arg, str) else arg.decode("latin-1"))
        elif name in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8", "BYTEARRAY8"):
            stack.append(bytes(arg))
        elif name == "EMPTY_TUPLE":
            stack.append(())
        elif name == "EMPTY_LIST":
            stack.append([])
        elif name == "EMPTY_DICT":
            stack.append({})
        elif name in ("TUPLE1", "TUPLE2", "TUPLE3"):
            n = int(name[-1])
            items = tuple(stack[-n:])
            del stack[-n:]
            stack.append(items)
        elif name in ("TUPLE", "LIST", "DICT"):
            k = len(stack) - 1 - stack[::-1].index(_MARK)
            items = stack[k + 1:]
            del stack[k:]
            if name == "TUPLE":
                stack.append(tuple(items))
            elif name == "LIST":
                stack.append(list(items))
            else:
                stack.append({items[i]: items[i + 1] for i in range(0, len(items), 2)})
        elif name in ("MEMOIZE",):
            memo[len(memo)] = stack[-1]
        elif name in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[int(arg)] = stack[-1]
        elif name in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[int(arg)])
        elif name == "STACK_GLOBAL":
            nm = stack.pop()
            mod = stack.pop()
            stack.append(GlobalRef(mod, nm))
        elif name == "GLOBAL":
            mod, nm = arg.split(" ", 1)
            stack.append(GlobalRef(mod, nm))
        elif name in ("REDUCE", "NEWOBJ"):
            args = stack.pop()
            fn = stack.pop()
            if not isinstance(fn, GlobalRef):
                raise PickleDecodeError(f"{name} on non-global {type(fn).__name__}")
            stack.append(_lower(Call(fn, tuple(args))))
        elif name == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, Call):
                obj.state = state
                stack[-1] = _lower(obj)
            else:
                raise PickleDecodeError("BUILD on non-object")
        elif name == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif name == "SETITEMS":
            k = len(stack) - 1 - stack[::-1].index(_MARK)
            items = stack[k + 1:]
            del stack[k:]
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif name == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif name == "APPENDS":
            k = len(stack) - 1 - stack[::-1].index(_MARK)
            items = stack[k + 1:]
            del stack[k:]
            stack[-1].extend(items)
        elif name == "POP":
            stack.pop()
        elif name == "DUP":
            stack.append(stack[-1])
        else:
            raise PickleDecodeError(f"unsupported opcode {name}")
    if len(stack) != 1:
        raise PickleDecodeError("malformed pickle stream")
    return stack[0]


# ------------------------------------------------------------------------------------- encoder

_FRAME_TARGET = 64 * 1024  # pickle's protocol-4 frame size target (pickle._Framer)


class _Writer:
    """Protocol-4 opcode writer with pickle's framing: opcodes accumulate in a frame that is emitted
    as ``FRAME <len>`` once it reaches 64 KiB at an object boundary or at the end, and a bytes payload
    of >= 64 KiB is written OUTSIDE any frame after the current one is flushed -- what CPython's
    pickler (and so joblib.dump) produces, byte for byte."""

    def __init__(self) -> None:
        self.out = io.BytesIO()
        self.frame = io.BytesIO()
        self.memo_n = 0

    def op(self, code: bytes, payload: bytes = b"") -> None:
        self.frame.write(code + payload)

    def commit(self, force: bool = False) -> None:
        n = self.frame.tell()
        if n and (force or n >= _FRAME_TARGET):
            # pickle._Framer.commit_frame: frames shorter than _FRAME_SIZE_MIN (4) go out without a header
            head = b"\x95" + struct.pack("<Q", n) if n >= 4 else b""
            self.out.write(head + self.frame.getvalue())  # FRAME
            self.frame = io.BytesIO()

    def large(self, header: bytes, payload: bytes) -> None:
        self.commit(force=True)
        self.out.write(header)
        self.out.write(payload)

    def getvalue(self) -> bytes:
        self.commit(force=True)
        return self.out.getvalue()

    def memoize(self) -> None:
        self.op(b"\x94")  # MEMOIZE
        self.memo_n += 1

    def str(self, s: str) -> None:
        self.commit()
        e = s.encode("utf-8")
        if len(e) < 256:
            self.op(b"\x8c", bytes([len(e)]) + e)  # SHORT_BINUNICODE
        else:
            self.op(b"X", struct.pack("<I", len(e)) + e)  # BINUNICODE
        self.memoize()

    def glob(self, mod: str, name: str) -> None:
        self.str(mod)
        self.str(name)
        self.op(b"\x93")  # STACK_GLOBAL
        self.memoize()

    def value(self, v: Any) -> None:
        self.commit()
        if v is None:
            self.op(b"N")
        elif v is True:
            self.op(b"\x88")
        elif v is False:
            self.op(b"\x89")
        elif isinstance(v, np.floating) and v.dtype == np.float64:
            # numpy.core.multiarray.scalar(dtype('f8'), raw-bytes), as numpy pickles a float64 scalar
            self.glob("numpy.core.multiarray", "scalar")
            self.glob("numpy", "dtype")
            self.str("f8")
            self.op(b"\x89")
            self.op(b"\x88")
            self.op(b"\x87")  # TUPLE3
            self.memoize()
            self.op(b"R")  # REDUCE
            self.memoize()
            self.op(b"(")  # MARK
            self.op(b"K", bytes([3]))
            self.str("<")
            self.op(b"N")
            self.op(b"N")
            self.op(b"N")
            self.op(b"J", struct.pack("<i", -1))
            self.op(b"J", struct.pack("<i", -1))
            self.op(b"K", bytes([0]))
            self.op(b"t")  # TUPLE
            self.memoize()
            self.op(b"b")  # BUILD
            raw = struct.pack("<d", float(v))
            self.op(b"C", bytes([len(raw)]) + raw)  # SHORT_BINBYTES
            self.memoize()
            self.op(b"\x86")  # TUPLE2
            self.memoize()
            self.op(b"R")
            self.memoize()
        elif isinstance(v, (bool, np.bool_)):
            self.op(b"\x88" if v else b"\x89")
        elif isinstance(v, (int, np.integer)):
            i = int(v)
            if 0 <= i < 256:
                self.op(b"K", bytes([i]))
            elif 0 <= i < 65536:
                self.op(b"M", struct.pack("<H", i))
            elif -2**31 <= i < 2**31:
                self.op(b"J", struct.pack("<i", i))
            else:
                raise ValueError("integer out of range for checkpoint writer")
        elif isinstance(v, (float, np.floating)):
            self.op(b"G", struct.pack(">d", float(v)))
        elif isinstance(v, str):
            self.str(v)
        elif isinstance(v, dict):
            self.op(b"}")
            self.memoize()
            if len(v) == 1:
                (k, x), = v.items()
                self.value(k)
                self.value(x)
                self.op(b"s")  # SETITEM (pickle uses it for one-item dicts)
            elif v:
                self.op(b"(")
                for k, x in v.items():
                    self.value(k)
                    self.value(x)
                self.op(b"u")  # SETITEMS
        else:
            raise ValueError(f"checkpoint writer cannot encode {type(v).__name__}")

    def bytearray(self, raw: bytes) -> None:
        self.glob("builtins", "bytearray")
        self.commit()
        head = b"B" + struct.pack("<I", len(raw)) if len(raw) < 2**32 else b"\x8e" + struct.pack("<Q", len(raw))
        if len(raw) >= _FRAME_TARGET:
            self.large(head, bytes(raw))  # BINBYTES / BINBYTES8 outside the frames
        else:
            self.op(head, bytes(raw))
        self.memoize()
        self.op(b"\x85")  # TUPLE1
        self.memoize()
        self.op(b"R")
        self.memoize()


def encode_xgb_classifier(state: dict[str, Any], booster_raw: bytes) -> bytes:
    """Pickle (protocol 4) an ``xgboost.sklearn.XGBClassifier`` with ``state`` and a UBJSON booster."""
    w = _Writer()
    w.out.write(b"\x80" + bytes([4]))  # PROTO 4 (before the first frame)
    w.glob("xgboost.sklearn", "XGBClassifier")
    w.op(b")")  # EMPTY_TUPLE
    w.op(b"\x81")  # NEWOBJ
    w.memoize()
    w.op(b"}")
    w.memoize()
    w.op(b"(")
    for k, v in state.items():
        w.value(k)
        w.value(v)
    w.value("_Booster")
    w.glob("xgboost.core", "Booster")
    w.op(b")")
    w.op(b"\x81")
    w.memoize()
    w.op(b"}")
    w.memoize()
    w.value("handle")
    w.bytearray(booster_raw)
    w.op(b"s")  # SETITEM
    w.op(b"b")  # BUILD (Booster)
    w.op(b"u")  # SETITEMS
    w.op(b"b")  # BUILD (XGBClassifier)
    w.op(b".")  # STOP
    return w.getvalue()


def read_xgb_classifier_pickle(data: bytes) -> tuple[dict[str, Any], bytes]:
    """Return (sklearn state dict without ``_Booster``, UBJSON booster bytes) from a checkpoint."""
    obj = decode(data)
    if not isinstance(obj, Call) or obj.func.qualname != "xgboost.sklearn.XGBClassifier":
        raise PickleDecodeError("not an xgboost.sklearn.XGBClassifier pickle")
    st = dict(obj.state or {})
    bst = st.pop("_Booster", None)
    if not isinstance(bst, Call) or bst.func.qualname != "xgboost.core.Booster":
        raise PickleDecodeError("checkpoint has no xgboost.core.Booster")
    raw = (bst.state or {}).get("handle")
    if not isinstance(raw, (bytes, bytearray)):
        raise PickleDecodeError("Booster.handle is not a bytearray")
    for k, v in list(st.items()):
        if isinstance(v, float) and math.isnan(v):
            st[k] = float("nan")
    return st, bytes(raw)
