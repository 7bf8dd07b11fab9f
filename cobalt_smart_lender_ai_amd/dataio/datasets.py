"""Raw-data acquisition and versioning (reference: data/download_data.py, the DVC pointers under
data/1-raw/lending-club-2007-2020Q3/*.dvc and .dvc/config).

* ``download_data`` -- the reference pulls a Google-Drive folder with ``gdown``; the same call is
  made when gdown is importable (no network on the build hosts: it then fails with a clear message).
* ``RAW_MANIFEST`` / ``verify`` -- the DVC-tracked raw files with their md5 and size; ``verify`` checks
  local copies (streamed md5, constant memory) the way ``dvc status`` would.
* ``stage_into_store`` -- copies a verified local raw file to the artifact store under the key the
  cleaning stage reads (``dataset/1-raw/...``).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass
from pathlib import Path

from ..config import RAW_DATA_KEY_FULL, RAW_DATA_KEY_SAMPLE

DRIVE_URL = "https://drive.google.com/drive/folders/1I1QSqJOSrkC4rGYvFKQsHxxDh7zUGcV_?usp=drive_link"
DVC_REMOTE = "s3://cobalt-lending-ai-data-lake/dataset"


@dataclass(frozen=True)
class RawFile:
    path: str
    md5: str
    size: int
    store_key: str


RAW_MANIFEST = (
    RawFile("data/1-raw/lending-club-2007-2020Q3/Loan_status_2007-2020Q3-100ksample.csv",
            "4e01f7e3ef869a35b65c400d3edda715", 73_991_891, RAW_DATA_KEY_SAMPLE),
    RawFile("data/1-raw/lending-club-2007-2020Q3/Loan_status_2007-2020Q3.gzip",
            "65adade308f21d60b7213088a88e684d", 1_773_470_505, RAW_DATA_KEY_FULL),
)


def md5_file(path: str | Path, block: int = 1 << 22) -> str:
    h = hashlib.md5()
    with open(path, "rb") as fh:
        while chunk := fh.read(block):
            h.update(chunk)
    return h.hexdigest()


def verify(root: str | Path = ".", files=RAW_MANIFEST) -> dict[str, str]:
    """{path: "ok" | "missing" | "size mismatch" | "md5 mismatch"}."""
    out = {}
    for f in files:
        p = Path(root) / f.path
        if not p.exists():
            out[f.path] = "missing"
        elif p.stat().st_size != f.size:
            out[f.path] = "size mismatch"
        else:
            out[f.path] = "ok" if md5_file(p) == f.md5 else "md5 mismatch"
    return out


def download_data(output: str = "data/all_data.zip", url: str = DRIVE_URL, quiet: bool = False) -> str:
    try:
        import gdown
    except ImportError as e:  # pragma: no cover - depends on the host
        raise RuntimeError("gdown is not installed; download the LendingClub files manually into "
                           "data/1-raw/lending-club-2007-2020Q3/ (see RAW_MANIFEST) or use `cli synth`") from e
    Path(output).parent.mkdir(parents=True, exist_ok=True)
    return gdown.download(url, output, quiet=quiet)


def stage_into_store(store, root: str | Path = ".", files=RAW_MANIFEST, check: bool = True) -> list[str]:
    """Upload verified local raw files to the artifact store keys the cleaning stage reads."""
    staged = []
    status = verify(root, files) if check else {f.path: "ok" for f in files}
    for f in files:
        if status.get(f.path) == "ok":
            store.upload_file(Path(root) / f.path, f.store_key)
            staged.append(f.store_key)
    return staged
