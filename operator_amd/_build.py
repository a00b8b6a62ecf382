"""In-tree native build for operator_amd (no pip install, no JIT cache).

Produces two shared objects next to this file:

* ``_C.*.so``        — the gfx950 HIP kernels (csrc/kernels/*.hip, compiled by
  ``hipcc --offload-arch=gfx950``) + torch bindings (csrc/*.cpp, g++ against
  the installed PyTorch-ROCm headers). Linked with an rpath to torch/lib first
  so the process has exactly one HIP runtime (torch's ``libamdhip64.so.7``).
* ``_patterns.*.so`` — the CPU pattern compiler / log packer / scorer
  (csrc/patterns/*.cpp, pybind11, no HIP or torch dependency).

Objects are cached under ``build/`` and rebuilt when a source or any header
under csrc/ is newer. ``python -m operator_amd._build`` builds both.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
PKG = ROOT / "operator_amd"
ARCH = os.environ.get("OAMD_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _newest_header_mtime() -> float:
    hs = glob.glob(str(CSRC / "**" / "*.h"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _stale(obj: Path, src: Path, hdr_mtime: float) -> bool:
    if not obj.exists():
        return True
    m = obj.stat().st_mtime
    return m < src.stat().st_mtime or m < hdr_mtime


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    libdirs = ce.library_paths(device_type="cuda")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    return inc, libdirs, abi, torch_lib


def build_patterns(verbose: bool = False, force: bool = False, out_dir: Path | None = None,
                   sanitize: bool | None = None) -> Path:
    """Host C++ module. ``sanitize`` (default: $OAMD_SANITIZE) adds ASan + UBSan —
    build it into ``out_dir`` and load it with libasan preloaded (tests/test_sanitizers.py)."""
    import pybind11

    out = (Path(out_dir) if out_dir else PKG) / f"_patterns{_ext_suffix()}"
    sanitize = bool(os.environ.get("OAMD_SANITIZE")) if sanitize is None else sanitize
    srcs = sorted((CSRC / "patterns").glob("*.cpp"))
    hdr = _newest_header_mtime()
    if not force and out.exists() and all(out.stat().st_mtime >= s.stat().st_mtime for s in srcs) \
            and out.stat().st_mtime >= hdr:
        return out
    cmd = [CXX, "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-pthread",
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{CSRC}",
           *map(str, srcs), "-o", str(out)]
    if sanitize:
        cmd[1:1] = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g", "-O1"]
    _run(cmd, verbose)
    return out


def build_kernels(verbose: bool = False, force: bool = False, jobs: int | None = None) -> Path:
    inc, libdirs, abi, torch_lib = _torch_flags()
    BUILD.mkdir(parents=True, exist_ok=True)
    hdr = _newest_header_mtime()
    hip_srcs = sorted((CSRC / "kernels").glob("*.hip"))
    cpp_srcs = sorted(CSRC.glob("*.cpp"))
    jobs = jobs or min(16, os.cpu_count() or 4)
    defs = [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
            "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1"]
    pyinc = f"-I{sysconfig.get_paths()['include']}"

    tasks = []
    objs = []
    for s in hip_srcs:
        o = BUILD / (s.stem + ".hip.o")
        objs.append(o)
        if force or _stale(o, s, hdr):
            tasks.append([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", str(s),
                          f"-I{CSRC / 'kernels'}", "-munsafe-fp-atomics", "-o", str(o)])
    for s in cpp_srcs:
        o = BUILD / (s.stem + ".cpp.o")
        objs.append(o)
        if force or _stale(o, s, hdr):
            tasks.append([CXX, "-O2", "-std=c++17", "-fPIC", "-c", str(s), f"-I{CSRC}", pyinc,
                          *[f"-isystem{i}" for i in inc], *defs, "-Wno-deprecated-declarations", "-o", str(o)])
    if tasks:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda c: _run(c, verbose), tasks))
    out = PKG / f"_C{_ext_suffix()}"
    if force or tasks or not out.exists() or any(out.stat().st_mtime < o.stat().st_mtime for o in objs):
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(out),
                f"-Wl,-rpath,{torch_lib}", f"-L{torch_lib}",
                *[f"-L{d}" for d in libdirs if d != torch_lib],
                "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64"]
        _run(link, verbose)
        _check_stubs(out)
    return out


def _check_stubs(so: Path) -> None:
    """Fail the build when a kernel's host launch stub is missing from the library: hipcc's
    host pass can drop one silently (a template kernel whose body its host-side semantic check
    rejects without a diagnostic), which otherwise only surfaces as an undefined symbol when
    the GPU box imports the module."""
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    r = subprocess.run([nm, "-u", str(so)], capture_output=True, text=True)
    missing = [ln.split()[-1] for ln in r.stdout.splitlines() if "__device_stub__" in ln]
    if missing:
        so.unlink(missing_ok=True)
        raise RuntimeError(f"native build: {len(missing)} kernel launch stub(s) undefined in {so.name}: {missing[:4]}")


def build(verbose: bool = False, force: bool = False) -> list[Path]:
    """Compile every native component for gfx950 (CPU-only host; hipcc cross-compiles)."""
    if shutil.which(HIPCC) is None and not os.path.exists(HIPCC):
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    return [build_patterns(verbose, force), build_kernels(verbose, force)]


if __name__ == "__main__":
    v = "-v" in sys.argv
    f = "-f" in sys.argv or "--force" in sys.argv
    # --host-only: just the host C++ pattern module (no ROCm needed): the multi-arch
    # controller image (docker/Dockerfile.controller), whose engines are remote or CPU
    for p in ([build_patterns(v, f)] if "--host-only" in sys.argv else build(verbose=v, force=f)):
        print(p)
