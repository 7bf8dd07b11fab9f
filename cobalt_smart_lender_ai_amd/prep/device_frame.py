"""Columnar, device-resident frame for the full-scale preprocessing pipeline.

The reference cleans ~2.9M rows x 143 columns with pandas (src/data_preprocessing/clean_data.py:87-158,
feature_engineering.py:44-184). Here the raw CSV is parsed ONCE on the host into a
:class:`DeviceFrame` whose columns all live in HBM, and stage 1 -> stage 2 -> feature engineering ->
the GBDT's quantile binning run on the GPU; only an artifact CSV write returns to the host.

* numeric columns: float64 ``[N]`` (NaN = missing) -- pandas' float64 / int64 values;
* string columns: int32 dictionary codes ``[N]`` (-1 = missing) + a host vocabulary. CSV parsing and
  dictionary encoding happen in pyarrow's C++ reader (K8/K10); every later string operation of the
  reference (``str.replace(" months")``, ``%`` stripping, ``\\d+`` extraction, ``%b-%Y`` dates,
  ``fillna("No Hardship")``, the ``loan_status`` map, sorted dummy levels, ``LabelEncoder``) runs once
  per DISTINCT value on the host and becomes a device gather over the codes;
* flag columns: uint8 ``[N]`` (dummies and ``_NA`` indicators).

Row filters compact every column on the device with one gather per column block
(:meth:`DeviceFrame.take`, K2), duplicate detection hashes whole rows on the device (K9), null counts
and per-row null counts are device reductions (K1/K2).
"""
from __future__ import annotations

from dataclasses import dataclass, replace

import numpy as np
import pandas as pd
import torch

from ..ops import prep_ops

# pandas.read_csv's default missing-value strings (the reference reads every CSV with pandas)
PANDAS_NA = ["", "#N/A", "#N/A N/A", "#NA", "-1.#IND", "-1.#QNAN", "-NaN", "-nan", "1.#IND", "1.#QNAN", "<NA>",
             "N/A", "NA", "NULL", "NaN", "None", "n/a", "nan", "null"]


@dataclass
class DCol:
    kind: str                 # "f" float64 values, "c" int32 dictionary codes (-1 = missing), "b" uint8 flags,
                              # "h" int64 device hashes of a near-unique string column (0 = missing)
    data: torch.Tensor        # [N] on the frame's device
    dtype: str                # pandas dtype on export: "float64" | "int64" | "bool" | "object" | "boolnull"
                              # (a true/false column with missing values: 1 / 0 / NaN on the device, object
                              # True / False / NaN in pandas, as pandas.read_csv types it)
    vocab: list | None = None  # "c": code -> value
    src: object = None        # "h": the ORIGINAL rows' text (host Arrow column, or csv_gpu.DeviceStrings in
                              # HBM), decoded lazily through rowid

    def null_mask(self) -> torch.Tensor:
        if self.kind == "f":
            return torch.isnan(self.data)
        if self.kind == "c":
            return self.data < 0
        if self.kind == "h":
            return self.data == 0
        return torch.zeros_like(self.data, dtype=torch.bool)

    @property
    def numeric(self) -> bool:  # pandas is_numeric_dtype
        return self.kind in ("f", "b")


class DeviceFrame:
    """Ordered columns of equal length on one device (see module doc)."""

    def __init__(self, cols: dict[str, DCol], n: int, device: torch.device, rowid: torch.Tensor | None = None):
        self.cols = dict(cols)
        self.n = int(n)
        self.device = torch.device(device)
        # original (ingest) row of every row -- lets hashed string columns be decoded lazily
        self.rowid = rowid if rowid is not None else torch.arange(self.n, device=self.device)

    # ------------------------------------------------------------------ structure
    @property
    def columns(self) -> list[str]:
        return list(self.cols)

    @property
    def shape(self) -> tuple[int, int]:
        return self.n, len(self.cols)

    def __len__(self) -> int:
        return self.n

    def __contains__(self, name: str) -> bool:
        return name in self.cols

    def __getitem__(self, name: str) -> DCol:
        return self.cols[name]

    def copy(self) -> "DeviceFrame":
        return DeviceFrame(self.cols, self.n, self.device, self.rowid)

    def drop(self, names, errors: str = "ignore") -> "DeviceFrame":
        names = [names] if isinstance(names, str) else list(names)
        if errors == "raise":
            miss = [c for c in names if c not in self.cols]
            if miss:
                raise KeyError(f"{miss} not found in axis")
        s = set(names)
        return DeviceFrame({k: v for k, v in self.cols.items() if k not in s}, self.n, self.device, self.rowid)

    def assign(self, **cols: DCol) -> "DeviceFrame":
        """DataFrame.assign: an existing name keeps its position, a new one is appended."""
        out = dict(self.cols)
        out.update(cols)
        return DeviceFrame(out, self.n, self.device, self.rowid)

    def host_strings(self, name: str, rows: torch.Tensor | None = None):
        """Values of a hashed ("h") string column for the current rows (or ``rows`` of them)."""
        import pyarrow.compute as pc

        c = self.cols[name]
        rid = self.rowid if rows is None else self.rowid[rows]
        if hasattr(c.src, "arrow"):  # GPU-ingested text (csv_gpu.DeviceStrings, in HBM): only these rows move
            return c.src.take(rid)
        return pc.take(c.src, rid.cpu().numpy())

    def as_categorical(self, name: str) -> DCol:
        """A string column as dictionary codes ("c"); a hashed column is decoded + encoded on demand."""
        import pyarrow.compute as pc

        c = self.cols[name]
        if c.kind != "h":
            return c
        enc = pc.dictionary_encode(self.host_strings(name))
        enc = enc.unify_dictionaries() if hasattr(enc, "unify_dictionaries") else enc
        chunks = enc.chunks if hasattr(enc, "chunks") else [enc]
        vocab = chunks[0].dictionary.to_pylist() if chunks else []
        idx = np.concatenate([ch.indices.fill_null(-1).to_numpy(zero_copy_only=False).astype(np.int32)
                              for ch in chunks] + [np.zeros(0, np.int32)])
        return DCol("c", torch.from_numpy(idx).to(self.device), "object", vocab)

    # ------------------------------------------------------------------ ingest / export
    @classmethod
    def from_arrow(cls, table, device, hash_unique_share: float = 0.2) -> "DeviceFrame":
        """Upload an Arrow table. String columns whose first 20k values are more than
        ``hash_unique_share`` distinct are hashed on the device (kind "h") instead of dictionary-encoded
        on the host (a near-unique column costs ~2 s per million rows to encode, ~1 ms to hash)."""
        import pyarrow as pa
        import pyarrow.compute as pc

        from ..ops import prep_ops as _po

        dev = torch.device(device)
        n = table.num_rows
        cols: dict[str, DCol] = {}
        for name, col in zip(table.column_names, table.columns):
            t = col.type
            if (pa.types.is_string(t) or pa.types.is_large_string(t)) and n >= 1000:
                head = col.slice(0, min(n, 20_000))
                if pc.count_distinct(head).as_py() > hash_unique_share * len(head):
                    cols[name] = DCol("h", _po.string_hash(col, dev), "object", src=col)
                    continue
            if pa.types.is_string(t) or pa.types.is_large_string(t) or pa.types.is_dictionary(t):
                enc = col if pa.types.is_dictionary(t) else pc.dictionary_encode(col)
                enc = enc.unify_dictionaries() if hasattr(enc, "unify_dictionaries") else enc
                chunks = enc.chunks if hasattr(enc, "chunks") else [enc]
                vocab = chunks[0].dictionary.to_pylist() if chunks else []
                idx = np.concatenate([c.indices.fill_null(-1).to_numpy(zero_copy_only=False).astype(np.int32)
                                      for c in chunks] + [np.zeros(0, np.int32)])
                cols[name] = DCol("c", torch.from_numpy(idx).to(dev), "object", vocab)
            elif pa.types.is_boolean(t) and col.null_count == 0:
                a = col.to_numpy(zero_copy_only=False).astype(np.uint8)
                cols[name] = DCol("b", torch.from_numpy(a).to(dev), "bool")
            elif pa.types.is_boolean(t):
                a = np.array(col.cast(pa.float64()).to_numpy(zero_copy_only=False), dtype=np.float64)
                cols[name] = DCol("f", torch.from_numpy(a).to(dev), "boolnull")
            elif pa.types.is_null(t):
                cols[name] = DCol("f", torch.full((n,), float("nan"), dtype=torch.float64, device=dev), "float64")
            else:
                is_int = pa.types.is_integer(t) and col.null_count == 0
                a = np.array(col.cast(pa.float64()).to_numpy(zero_copy_only=False), dtype=np.float64)  # writable
                cols[name] = DCol("f", torch.from_numpy(a).to(dev),
                                  "int64" if is_int else "float64")
        return cls(cols, n, dev)

    @classmethod
    def read_csv(cls, path_or_bytes, device, threads: bool = True, engine: str = "auto",
                 timings: dict | None = None, float_precision: str = "round_trip") -> "DeviceFrame":
        """Parse a (optionally gzipped) CSV with pandas' missing values into device columns.

        ``engine="gpu"`` (the default on a GPU device, ``"auto"``): the bytes go to HBM and the
        tokenizer / parser / dictionary encoder of ``csrc/csv.hip`` run there (prep/csv_gpu.py); a file
        it cannot lay out as a rectangle falls back to ``"arrow"``: pyarrow's multithreaded C++ reader
        on the host, then every column is uploaded. ``float_precision="high"`` reproduces pandas'
        default float conversion (GPU engine only: the Arrow reader rounds correctly)."""
        import io

        import pyarrow as pa
        import pyarrow.csv as pcsv

        if engine not in ("auto", "gpu", "arrow"):
            raise ValueError(f"engine must be auto, gpu or arrow, got {engine!r}")
        if float_precision == "high" and (engine == "arrow" or torch.device(device).type != "cuda"):
            raise ValueError('float_precision="high" needs the GPU engine')
        if engine in ("auto", "gpu") and torch.device(device).type == "cuda":
            from .csv_gpu import CsvLayoutError, read_csv_gpu

            try:
                return read_csv_gpu(path_or_bytes, device, timings=timings, float_precision=float_precision)
            except CsvLayoutError:
                if engine == "gpu" or float_precision == "high":
                    raise

        src = path_or_bytes
        if isinstance(src, (bytes, bytearray)):
            src = pa.BufferReader(bytes(src)) if src[:2] != b"\x1f\x8b" else pa.CompressedInputStream(
                pa.BufferReader(bytes(src)), "gzip")
        elif str(src).endswith(".gz") or str(src).endswith(".gzip"):
            src = pa.CompressedInputStream(pa.OSFile(str(src)), "gzip")
        tab = pcsv.read_csv(src, read_options=pcsv.ReadOptions(use_threads=threads, block_size=1 << 26),
                            convert_options=pcsv.ConvertOptions(strings_can_be_null=True, null_values=PANDAS_NA,
                                                                quoted_strings_can_be_null=True))
        from .csv_gpu import dedup_names

        if len(set(tab.column_names)) != len(tab.column_names):  # repeated headers: pandas' a, a.1, ...
            tab = tab.rename_columns(dedup_names(tab.column_names))
        _ = io
        return cls.from_arrow(tab, device)

    @classmethod
    def from_pandas(cls, df: pd.DataFrame, device) -> "DeviceFrame":
        import pyarrow as pa

        return cls.from_arrow(pa.Table.from_pandas(df, preserve_index=False), device)

    def to_pandas(self) -> pd.DataFrame:
        out = {}
        for name, c in self.cols.items():
            if c.kind == "h":
                out[name] = pd.Series(self.host_strings(name).to_pandas(), dtype=object).where(
                    lambda v: v.notna(), np.nan)
                continue
            a = c.data.cpu().numpy()
            if c.kind == "c":
                voc = np.array(list(c.vocab) + [np.nan], dtype=object)
                out[name] = pd.Series(voc[np.where(a < 0, len(c.vocab), a)], dtype=object)
            elif c.kind == "b":
                out[name] = a.astype(bool) if c.dtype == "bool" else a.astype(np.int64)
            elif c.dtype == "boolnull":
                v = np.empty(len(a), dtype=object)
                v[:] = a == 1.0
                v[np.isnan(a)] = np.nan
                out[name] = v
            elif c.dtype == "int64" and not np.isnan(a).any():
                out[name] = a.astype(np.int64)
            else:
                out[name] = a
        return pd.DataFrame(out, columns=self.columns)

    def matrix(self, names: list[str], dtype=torch.float32) -> torch.Tensor:
        """Row-major ``[N, len(names)]`` device matrix of numeric / flag columns (the GBDT input)."""
        out = torch.empty((self.n, len(names)), dtype=dtype, device=self.device)
        for j, nm in enumerate(names):
            c = self.cols[nm]
            if c.kind == "c":
                raise TypeError(f"column {nm!r} is not numeric")
            out[:, j] = c.data.to(dtype)
        return out

    # ------------------------------------------------------------------ nulls / rows
    def _null_block(self, names: list[str]) -> torch.Tensor:
        """[C, N] float64 block whose NaNs are the columns' missing values (input of the K1/K2 kernels)."""
        blk = torch.empty((len(names), self.n), dtype=torch.float64, device=self.device)
        for i, nm in enumerate(names):
            c = self.cols[nm]
            if c.kind == "f":
                blk[i] = c.data
            else:
                blk[i] = torch.where(c.null_mask(), float("nan"), 0.0)
        return blk

    def null_counts(self) -> dict[str, int]:
        """``df.isnull().sum()`` (K1 kernel, one host sync)."""
        names = self.columns
        if not names or self.n == 0:
            return {k: 0 for k in names}
        cnt = prep_ops.col_null_counts(self._null_block(names)).cpu().numpy()
        return dict(zip(names, cnt.tolist()))

    def row_null_counts(self, names: list[str] | None = None) -> torch.Tensor:
        """Per-row missing count over ``names`` (default all columns; K2 kernel), int32 [N]."""
        names = self.columns if names is None else [c for c in self.columns if c in set(names)]
        if not names:
            return torch.zeros(self.n, dtype=torch.int32, device=self.device)
        return prep_ops.row_null_counts(self._null_block(names))

    def take(self, keep: torch.Tensor) -> "DeviceFrame":
        """Rows where ``keep`` (bool [N]) is true, order preserved (K2 stream compaction): one index
        vector, then one gather per column block (float64 / int32 / uint8)."""
        idx = keep.nonzero().squeeze(1)
        m = int(idx.numel())
        if m == self.n:
            return self.copy()
        rowid = self.rowid.index_select(0, idx)
        out = {}
        groups: dict[str, list[str]] = {}
        for nm, c in self.cols.items():
            groups.setdefault(c.kind, []).append(nm)
        for kind, names in groups.items():
            blk = torch.stack([self.cols[nm].data for nm in names])  # [C, N]
            g = blk.index_select(1, idx)
            for i, nm in enumerate(names):
                out[nm] = replace(self.cols[nm], data=g[i])
        return DeviceFrame({nm: out[nm] for nm in self.cols}, m, self.device, rowid)

    def duplicated(self) -> torch.Tensor:
        """``df.duplicated(keep='first')`` over all columns: device row hash + sort + exact pairwise
        verification (K9). Codes compare exactly as their strings (one vocabulary per column)."""
        if self.n == 0:
            return torch.zeros(0, dtype=torch.bool, device=self.device)
        rows = []
        for c in self.cols.values():
            if c.kind == "c":
                rows.append(torch.where(c.data < 0, float("nan"), c.data.to(torch.float64)))
            elif c.kind == "h":  # two exact 32-bit halves of the hash
                rows.append((c.data & 0xFFFFFFFF).to(torch.float64))
                rows.append((c.data >> 32).to(torch.float64))
            else:
                rows.append(c.data.to(torch.float64))
        dup, (a, b) = prep_ops.duplicated_numeric(torch.stack(rows))
        hashed = [nm for nm, c in self.cols.items() if c.kind == "h"]
        if hashed and a.numel():  # hashes stand in for strings: verify candidate pairs exactly
            for nm in hashed:
                sa = self.host_strings(nm, a).to_pylist()
                sb = self.host_strings(nm, b).to_pylist()
                bad = [k for k, (x, y) in enumerate(zip(sa, sb)) if x != y]
                if bad:
                    dup[b[torch.tensor(bad, device=b.device)]] = False
        return dup


def gather_vocab(col: DCol, table: np.ndarray, fill: float = float("nan")) -> torch.Tensor:
    """Per-row float64 values of a per-DISTINCT-value lookup ``table`` ([len(vocab)]); missing -> fill."""
    t = torch.from_numpy(np.append(np.asarray(table, dtype=np.float64), fill)).to(col.data.device)
    idx = torch.where(col.data < 0, len(table), col.data.long())
    return t[idx]
