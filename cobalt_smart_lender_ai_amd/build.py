"""In-tree build of the native library ``_lib/libcobalt_hip.so`` (HIP kernels for gfx950 + C++ runtime).

Every ``csrc/*.hip`` is compiled with ``hipcc --offload-arch=gfx950`` and every ``csrc/*.cpp`` as host
C++; the objects are linked into one shared library that Python binds with ``ctypes``
(see ``_native.py``). The library links against the HIP runtime that PyTorch-ROCm ships
(``torch/lib/libamdhip64.so``) so a process never holds two HIP runtimes.

Usage: ``python -m cobalt_smart_lender_ai_amd.build [--force] [-j N] [--sanitize]``.

``--sanitize`` builds ``_lib/libcobalt_hip_asan.so``: the same library with the HOST code compiled
under AddressSanitizer + UndefinedBehaviorSanitizer (``-Xarch_host -fsanitize=...``; device code
is not instrumented -- GPU ASan / XNACK are not available on MI355X pools). Use it on a development
host with the ASan runtime preloaded (``LD_PRELOAD=$(hipcc -print-file-name=libclang_rt.asan-x86_64.so)``,
``COBALT_NATIVE_LIB=<path>``); pair it with ``AMD_SERIALIZE_KERNEL=3`` / ``HIP_LAUNCH_BLOCKING=1`` to
serialise launches when chasing a fault. The race oracle of the normal build is
determinism: exact integer histograms, fixed reduction orders, bit-identical repeat/oracle tests.
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
from .config import knob

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
OUT_DIR = PKG_DIR / "_lib"
LIB_NAME = "libcobalt_hip.so"
ARCH = knob("COBALT_OFFLOAD_ARCH", "gfx950")

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


SANITIZE_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                  "-Xarch_host", "-fno-omit-frame-pointer", "-g"]


def compile_cmd(src: Path, obj: Path, sanitize: bool = False) -> list[str]:
    extra = SANITIZE_FLAGS if sanitize else []
    if src.suffix == ".hip":
        return [HIPCC, f"--offload-arch={ARCH}", *COMMON_FLAGS, *extra, "-c", str(src), "-o", str(obj)]
    return [HIPCC, *COMMON_FLAGS, *extra, "-c", str(src), "-o", str(obj)]


def _compile(src: Path, obj: Path, sanitize: bool = False) -> tuple[Path, str]:
    cmd = compile_cmd(src, obj, sanitize)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj, r.stderr


def build(force: bool = False, jobs: int | None = None, verbose: bool = False, sanitize: bool = False) -> Path:
    """Compile all sources (in parallel) and link ``_lib/libcobalt_hip.so`` (``sanitize``: the
    host-ASan/UBSan variant ``_lib/libcobalt_hip_asan.so``). Returns the library path."""
    if sanitize:
        return _build_sanitized(jobs)
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


def _build_sanitized(jobs: int | None) -> Path:
    obj_dir = OUT_DIR / "obj_asan"
    obj_dir.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=jobs or min(8, len(srcs))) as ex:
        objs = [f.result()[0] for f in [ex.submit(_compile, s, obj_dir / (s.name + ".o"), True) for s in srcs]]
    out = OUT_DIR / "libcobalt_hip_asan.so"
    link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Xarch_host", "-fsanitize=address",
            "-Xarch_host", "-fsanitize=undefined", "-shared-libasan", *[str(o) for o in objs], "-o", str(out), "-ldl"]
    torch_lib = _torch_lib_dir()
    if torch_lib:
        link += [f"-L{torch_lib}", f"-Wl,-rpath,{torch_lib}"]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(link)}\n{r.stdout}\n{r.stderr}")
    return out


def main(argv: list[str] | None = None) -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--sanitize", action="store_true", help="host ASan/UBSan variant (libcobalt_hip_asan.so)")
    a = ap.parse_args(argv)
    p = build(force=a.force, jobs=a.jobs, verbose=a.verbose, sanitize=a.sanitize)
    print(p)


if __name__ == "__main__":
    main()
