"""Every COBALT_* environment knob is registered and documented (config.KNOBS); the native library
reads its knobs only through its registry (csrc/knobs.cpp: the one getenv call site of csrc/)."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "cobalt_smart_lender_ai_amd"


def test_native_getenv_only_in_the_registry():
    calls = []
    for p in sorted((PKG / "csrc").glob("*")):
        for i, line in enumerate(p.read_text().splitlines(), 1):
            if "getenv(" in line and not line.lstrip().startswith("//"):
                calls.append(p.name)
    assert calls == ["knobs.cpp"], calls


def test_native_registry_names_are_documented():
    from cobalt_smart_lender_ai_amd.config import KNOBS

    src = (PKG / "csrc" / "knobs.cpp").read_text()
    table = src[src.index("kKnobNames"):src.index("};")]
    names = re.findall(r'"(COBALT_[A-Z0-9_]+)"', table)
    header = (PKG / "csrc" / "knobs.h").read_text()
    n_enum = len(re.findall(r"^\s+[A-Z][A-Za-z0-9]*,\s+// COBALT_", header, re.M))
    assert len(names) == n_enum == len(set(names)), (names, n_enum)
    for n in names:
        assert n in KNOBS and KNOBS[n].scope == "native", n


def test_every_knob_in_the_tree_is_registered():
    from cobalt_smart_lender_ai_amd.config import KNOBS

    seen = set()
    for base in (PKG, ROOT / "tests", ROOT / "src", ROOT / "bench.py", ROOT / "__graft_entry__.py"):
        files = [base] if base.is_file() else [p for p in base.rglob("*") if p.suffix in (".py", ".hip", ".cpp", ".h")]
        for p in files:
            seen |= set(re.findall(r"\bCOBALT_[A-Z][A-Z0-9_]*[A-Z0-9]\b", p.read_text()))
    # C/C++ identifiers that are not environment variables
    seen -= {"COBALT_API", "COBALT_IPC_ACQUIRE_FENCE", "COBALT_NOT_A_KNOB"}
    missing = sorted(n for n in seen if n not in KNOBS)
    assert not missing, missing
    for n, k in KNOBS.items():
        assert k.doc and k.scope in ("native", "python", "test"), n


def test_knob_lookup_refuses_unregistered_names():
    import pytest

    from cobalt_smart_lender_ai_amd.config import knob

    assert knob("COBALT_IPC_SLOT_MB", "64") is not None
    with pytest.raises(KeyError):
        knob("COBALT_NOT_A_KNOB")


def test_python_reads_knobs_through_the_registry():
    """The Python side reads COBALT_* variables only through config.knob() (which refuses unregistered
    names); direct os.environ reads remain only for the registry itself (writes -- e.g. cumask setting
    COBALT_CU_BUDGET for the native side -- are allowed)."""
    reads = []
    pat = re.compile(r'os\.environ\.get\("COBALT_|os\.environ\["COBALT_[A-Z0-9_]+"\](?!\s*=[^=])')
    for p in [*PKG.rglob("*.py"), ROOT / "bench.py", ROOT / "__graft_entry__.py"]:
        if p.name == "config.py" and p.parent == PKG:
            continue
        for i, line in enumerate(p.read_text().splitlines(), 1):
            if pat.search(line):
                reads.append(f"{p.relative_to(ROOT)}:{i}")
    assert not reads, reads
