"""Artifact / data-lake store with the reference's S3 key layout.

The reference moves every dataset and model through ``boto3`` against the bucket
``cobalt-lending-ai-data-lake`` (clean_data.py:44-84, feature_engineering.py:24-42,
model_tree_train_test.py:37-71, cobalt_fast_api.py:36-52). This module keeps the same keys behind a
small interface with two backends:

* ``LocalStore`` -- a directory whose layout mirrors the bucket (default; works offline);
* ``S3Store``    -- boto3, used only when importable and requested (``s3://bucket`` URIs).

``get_store()`` picks the backend from ``COBALT_ARTIFACT_URI`` (a local path or ``s3://bucket``).
"""
from __future__ import annotations

import io
import os
import shutil
from pathlib import Path

import pandas as pd

from ..config import BUCKET_NAME
from ..config import knob


class ArtifactStore:
    def get_bytes(self, key: str) -> bytes:
        raise NotImplementedError

    def put_bytes(self, key: str, data: bytes) -> None:
        raise NotImplementedError

    def exists(self, key: str) -> bool:
        raise NotImplementedError

    def download_file(self, key: str, path: str | Path) -> Path:
        p = Path(path)
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(self.get_bytes(key))
        return p

    def upload_file(self, path: str | Path, key: str) -> None:
        self.put_bytes(key, Path(path).read_bytes())

    # pandas helpers (the reference's read_csv / to_csv round trips)
    def read_csv(self, key: str, **kw) -> pd.DataFrame:
        data = self.get_bytes(key)
        comp = "gzip" if data[:2] == b"\x1f\x8b" else None
        return pd.read_csv(io.BytesIO(data), low_memory=False, compression=comp, **kw)

    def write_csv(self, df: pd.DataFrame, key: str) -> None:
        buf = io.StringIO()
        df.to_csv(buf, index=False)
        self.put_bytes(key, buf.getvalue().encode())

    def save_figure(self, fig, key: str) -> None:
        buf = io.BytesIO()
        fig.savefig(buf, format="png")
        self.put_bytes(key, buf.getvalue())


class LocalStore(ArtifactStore):
    def __init__(self, root: str | Path):
        self.root = Path(root)

    def _p(self, key: str) -> Path:
        p = (self.root / key.lstrip("/")).resolve()
        if self.root.resolve() not in p.parents and p != self.root.resolve():
            raise ValueError(f"key escapes the store root: {key}")
        return p

    def get_bytes(self, key: str) -> bytes:
        return self._p(key).read_bytes()

    def put_bytes(self, key: str, data: bytes) -> None:
        p = self._p(key)
        p.parent.mkdir(parents=True, exist_ok=True)
        tmp = p.with_name(p.name + ".tmp")
        tmp.write_bytes(data)
        os.replace(tmp, p)

    def exists(self, key: str) -> bool:
        return self._p(key).exists()

    def download_file(self, key: str, path: str | Path) -> Path:
        p = Path(path)
        p.parent.mkdir(parents=True, exist_ok=True)
        shutil.copyfile(self._p(key), p)
        return p


class S3Store(ArtifactStore):
    def __init__(self, bucket: str = BUCKET_NAME):
        try:
            import boto3  # noqa: F401
        except ImportError as e:  # pragma: no cover - boto3 is not installed in this image
            raise RuntimeError("S3 artifact store requested but boto3 is not installed") from e
        import boto3

        self.bucket = bucket
        self.client = boto3.client("s3")

    def get_bytes(self, key: str) -> bytes:  # pragma: no cover
        return self.client.get_object(Bucket=self.bucket, Key=key)["Body"].read()

    def put_bytes(self, key: str, data: bytes) -> None:  # pragma: no cover
        self.client.put_object(Bucket=self.bucket, Key=key,
                               Body=data if isinstance(data, (bytes, bytearray)) else bytes(data))

    def exists(self, key: str) -> bool:  # pragma: no cover
        try:
            self.client.head_object(Bucket=self.bucket, Key=key)
            return True
        except Exception:  # noqa: BLE001
            return False


def get_store(uri: str | None = None) -> ArtifactStore:
    uri = uri or knob("COBALT_ARTIFACT_URI", "data-lake")
    if uri.startswith("s3://"):
        return S3Store(uri[5:].split("/")[0] or BUCKET_NAME)
    return LocalStore(uri)
