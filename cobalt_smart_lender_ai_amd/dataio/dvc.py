"""DVC-compatible data versioning (reference: ``.dvc/config:1-4`` and the pointers
``data/1-raw/lending-club-2007-2020Q3/*.dvc``).

The reference versions its raw LendingClub files with DVC: a small YAML pointer next to each data
path records the file's md5 / size, and the content lives in an S3 remote
(``s3://cobalt-lending-ai-data-lake/dataset``). DVC itself is not a dependency here; this module
reads and writes the same pointer format and the same remote layout (DVC 3: ``files/md5/<2>/<30>``),
so ``dvc pull`` / ``dvc push`` of the reference repo and these functions interoperate:

* :func:`read_config` -- ``.dvc/config`` (core.remote, remote urls);
* :func:`read_pointer` / :func:`add` -- parse / write ``<file>.dvc`` (``outs: [{md5, size, hash, path}]``);
* :func:`status` -- ``ok`` / ``missing`` / ``modified`` (streamed md5, constant memory);
* :func:`push` / :func:`pull` -- content-addressed upload / download through any
  :class:`~.artifacts.ArtifactStore` (a local directory mirror of the remote, or S3), verified by md5.
"""
from __future__ import annotations

import re
import shutil
from dataclasses import dataclass
from pathlib import Path

import yaml

from .datasets import md5_file


@dataclass(frozen=True)
class Out:
    path: str       # relative to the pointer's directory
    md5: str
    size: int
    hash: str = "md5"


def read_config(repo_root: str | Path = ".") -> dict:
    """``.dvc/config`` (+ ``config.local``) as ``{"core": {...}, "remotes": {name: {"url": ...}}}``."""
    out: dict = {"core": {}, "remotes": {}}
    for name in ("config", "config.local"):
        p = Path(repo_root) / ".dvc" / name
        if not p.exists():
            continue
        sect = None
        for raw in p.read_text().splitlines():
            line = raw.strip()
            if not line or line.startswith(("#", ";")):
                continue
            m = re.fullmatch(r"\[\s*'?(.*?)'?\s*\]", line)
            if m:
                sect = m.group(1).strip()
                continue
            if "=" in line and sect is not None:
                k, v = (x.strip() for x in line.split("=", 1))
                rm = re.fullmatch(r'remote\s+"(.+)"', sect)
                if rm:
                    out["remotes"].setdefault(rm.group(1), {})[k] = v
                else:
                    out.setdefault(sect, {})[k] = v
    return out


def read_pointer(pointer: str | Path) -> list[Out]:
    data = yaml.safe_load(Path(pointer).read_text()) or {}
    return [Out(o["path"], str(o["md5"]), int(o["size"]), o.get("hash", "md5")) for o in data.get("outs", [])]


def add(data_path: str | Path) -> Path:
    """Write ``<data_path>.dvc`` (DVC 3 pointer) for a file; returns the pointer path."""
    p = Path(data_path)
    body = {"outs": [{"md5": md5_file(p), "size": p.stat().st_size, "hash": "md5", "path": p.name}]}
    ptr = p.with_name(p.name + ".dvc")
    ptr.write_text(yaml.safe_dump(body, sort_keys=False))
    return ptr


def _data_path(pointer: Path, out: Out) -> Path:
    return pointer.parent / out.path


def status(pointer: str | Path) -> dict[str, str]:
    """{data path: "ok" | "missing" | "modified"} for every output of a pointer."""
    ptr = Path(pointer)
    res = {}
    for o in read_pointer(ptr):
        p = _data_path(ptr, o)
        if not p.exists():
            res[str(p)] = "missing"
        elif p.stat().st_size != o.size or md5_file(p) != o.md5:
            res[str(p)] = "modified"
        else:
            res[str(p)] = "ok"
    return res


def cache_key(md5: str) -> str:
    """DVC 3 remote layout of a content hash."""
    return f"files/md5/{md5[:2]}/{md5[2:]}"


def push(pointer: str | Path, store, prefix: str = "") -> list[str]:
    """Upload each output's content under its content key (skips ones already in the remote)."""
    ptr = Path(pointer)
    keys = []
    for o in read_pointer(ptr):
        p = _data_path(ptr, o)
        if md5_file(p) != o.md5:
            raise ValueError(f"{p} does not match its pointer (run add() to re-version it)")
        key = prefix + cache_key(o.md5)
        if not (hasattr(store, "exists") and store.exists(key)):
            if hasattr(store, "upload_file"):
                store.upload_file(p, key)
            else:
                store.put_bytes(key, p.read_bytes())
        keys.append(key)
    return keys


def pull(pointer: str | Path, store, prefix: str = "") -> list[Path]:
    """Download each output by its content key next to the pointer and verify md5 + size."""
    ptr = Path(pointer)
    got = []
    for o in read_pointer(ptr):
        p = _data_path(ptr, o)
        tmp = p.with_name(p.name + ".part")
        key = prefix + cache_key(o.md5)
        if hasattr(store, "download_file"):
            store.download_file(key, tmp)
        else:
            tmp.parent.mkdir(parents=True, exist_ok=True)
            tmp.write_bytes(store.get_bytes(key))
        if tmp.stat().st_size != o.size or md5_file(tmp) != o.md5:
            tmp.unlink()
            raise ValueError(f"content of {key} does not match the pointer {ptr}")
        shutil.move(str(tmp), str(p))
        got.append(p)
    return got
