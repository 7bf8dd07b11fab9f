"""In-tree build of the native library ``_lib/libcobalt_hip.so`` (HIP kernels for gfx950 + C++ runtime).

Every ``csrc/*.hip`` is compiled with ``hipcc --offload-arch=gfx950`` and every ``csrc/*.cpp`` as host
C++; the objects are linked into one shared library that Python binds with ``ctypes``
(see ``_native.py``). The library links against the HIP runtime that PyTorch-ROCm ships
(``torch/lib/libamdhip64.so``) so a process never holds two HIP runtimes.

Usage: ``python -m cobalt_smart_lender_ai_amd.build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
OUT_DIR = PKG_DIR / "_lib"
LIB_NAME = "libcobalt_hip.so"
ARCH = os.environ.get("COBALT_OFFLOAD_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
COMMON_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
                "-Wno-unused-variable", "-Wno-unused-but-set-variable"]


def _torch_lib_dir() -> str:
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or spec.origin is None:
        return ""
    return str(Path(spec.origin).parent / "lib")


def sources() -> list[Path]:
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")))


def _digest() -> str:
    h = hashlib.sha256()
    for p in sorted(list(CSRC.glob("*")) + [Path(__file__)]):
        if p.is_file():
            h.update(p.name.encode())
            h.update(p.read_bytes())
    h.update(ARCH.encode())
    return h.hexdigest()


def lib_path() -> Path:
    return OUT_DIR / LIB_NAME


def is_stale() -> bool:
    stamp = OUT_DIR / (LIB_NAME + ".sha256")
    return not lib_path().exists() or not stamp.exists() or stamp.read_text().strip() != _digest()


def _compile(src: Path, obj: Path) -> tuple[Path, str]:
    if src.suffix == ".hip":
        cmd = [HIPCC, f"--offload-arch={ARCH}", *COMMON_FLAGS, "-c", str(src), "-o", str(obj)]
    else:
        cmd = [HIPCC, *COMMON_FLAGS, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj, r.stderr


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    """Compile all sources (in parallel) and link ``_lib/libcobalt_hip.so``. Returns the library path."""
    if not force and not is_stale():
        return lib_path()
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    obj_dir = OUT_DIR / "obj"
    obj_dir.mkdir(exist_ok=True)
    srcs = sources()
    jobs = jobs or min(8, max(1, os.cpu_count() or 1), len(srcs))
    objs: list[Path] = []
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, obj_dir / (s.name + ".o")) for s in srcs]
        for f in futs:
            obj, log = f.result()
            objs.append(obj)
            if verbose and log.strip():
                print(log, file=sys.stderr)
    torch_lib = _torch_lib_dir()
    link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *[str(o) for o in objs], "-o",
            str(OUT_DIR / (LIB_NAME + ".tmp")), "-ldl"]
    if torch_lib:
        link += [f"-L{torch_lib}", f"-Wl,-rpath,{torch_lib}"]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(link)}\n{r.stdout}\n{r.stderr}")
    os.replace(OUT_DIR / (LIB_NAME + ".tmp"), lib_path())
    (OUT_DIR / (LIB_NAME + ".sha256")).write_text(_digest())
    return lib_path()


def main(argv: list[str] | None = None) -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    p = build(force=a.force, jobs=a.jobs, verbose=a.verbose)
    print(p)


if __name__ == "__main__":
    main()
