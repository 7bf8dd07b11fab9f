"""DVC-compatible data versioning (reference: .dvc/config:1-4, data/1-raw/.../*.dvc)."""
from pathlib import Path

import pytest

from cobalt_smart_lender_ai_amd.dataio import datasets, dvc
from cobalt_smart_lender_ai_amd.dataio.artifacts import LocalStore

REF = Path("/root/reference")


def test_read_config_format(tmp_path):
    (tmp_path / ".dvc").mkdir()
    (tmp_path / ".dvc" / "config").write_text(
        "[core]\n    remote = myremote\n['remote \"myremote\"']\n    url = s3://cobalt-lending-ai-data-lake/dataset\n")
    cfg = dvc.read_config(tmp_path)
    assert cfg["core"]["remote"] == "myremote"
    assert cfg["remotes"]["myremote"]["url"] == datasets.DVC_REMOTE


def test_reference_pointers_match_the_manifest():
    ptrs = sorted(REF.glob("data/1-raw/lending-club-2007-2020Q3/*.dvc"))
    if not ptrs:
        pytest.skip("reference pointers not available")
    outs = {o.path: o for p in ptrs for o in dvc.read_pointer(p)}
    for f in datasets.RAW_MANIFEST:
        o = outs[Path(f.path).name]
        assert (o.md5, o.size, o.hash) == (f.md5, f.size, "md5")
    if (REF / ".dvc" / "config").exists():
        assert dvc.read_config(REF)["remotes"]["myremote"]["url"] == datasets.DVC_REMOTE


def test_add_status_push_pull_round_trip(tmp_path):
    data = tmp_path / "work" / "raw.csv"
    data.parent.mkdir()
    data.write_bytes(b"a,b\n1,2\n" * 1000)
    ptr = dvc.add(data)
    (o,) = dvc.read_pointer(ptr)
    assert o.path == "raw.csv" and o.size == data.stat().st_size and o.md5 == datasets.md5_file(data)
    assert dvc.status(ptr) == {str(data): "ok"}
    remote = LocalStore(tmp_path / "remote")
    (key,) = dvc.push(ptr, remote)
    assert key == f"files/md5/{o.md5[:2]}/{o.md5[2:]}" and remote.exists(key)
    data.write_bytes(b"tampered")
    assert dvc.status(ptr) == {str(data): "modified"}
    with pytest.raises(ValueError):
        dvc.push(ptr, remote)
    data.unlink()
    assert dvc.status(ptr) == {str(data): "missing"}
    dvc.pull(ptr, remote)
    assert dvc.status(ptr) == {str(data): "ok"}
    # a corrupted remote object is refused
    (tmp_path / "remote" / key).write_bytes(b"x")
    data.unlink()
    with pytest.raises(ValueError):
        dvc.pull(ptr, remote)
    assert not data.exists()
