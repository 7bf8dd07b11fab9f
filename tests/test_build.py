"""Native build plumbing: the host-sanitizer variant instruments host code only."""
import subprocess
from pathlib import Path

import pytest

from cobalt_smart_lender_ai_amd import build


@pytest.mark.skipif(not Path(build.HIPCC).exists(), reason="hipcc not installed")
def test_sanitizer_flags_instrument_host_code(tmp_path):
    src = build.CSRC / "comm.cpp"
    cmd = build.compile_cmd(src, tmp_path / "comm.o", sanitize=True)
    assert cmd.count("-Xarch_host") >= 2 and "-fsanitize=address" in cmd
    # every -fsanitize flag is scoped to the host compilation (no GPU ASan on this platform)
    for i, a in enumerate(cmd):
        if a.startswith("-fsanitize="):
            assert cmd[i - 1] == "-Xarch_host"
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    nm = subprocess.run(["nm", str(tmp_path / "comm.o")], capture_output=True, text=True).stdout
    assert "__asan" in nm
    plain = subprocess.run(build.compile_cmd(src, tmp_path / "plain.o"), capture_output=True, text=True)
    assert plain.returncode == 0
    assert "__asan" not in subprocess.run(["nm", str(tmp_path / "plain.o")], capture_output=True, text=True).stdout
