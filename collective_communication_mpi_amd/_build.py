"""In-tree build of the native extensions.

* ``_host``   : C++17 shared-memory host plane (g++; no GPU toolchain needed).
* ``_device`` : HIP/C++ device plane + CDNA4 kernels, compiled by ``hipcc
  --offload-arch=gfx950`` and linked against libamdhip64 / librccl.

Both land next to this file so they travel with the repo snapshot to the GPU
box.  Builds are incremental (mtime based) and serialised with a file lock so
that N ranks importing the package at once build it exactly once.

Usage: ``python -m collective_communication_mpi_amd._build [host|device|all] [--force]``
"""
from __future__ import annotations

import fcntl
import os
import shutil
import subprocess
import sys
import sysconfig
import tempfile
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("CCMPI_OFFLOAD_ARCH", "gfx950")


def _py_includes() -> list[str]:
    import pybind11

    inc = {sysconfig.get_paths()["include"], sysconfig.get_paths()["platinclude"], pybind11.get_include()}
    return [f"-I{p}" for p in sorted(inc)]


def host_target() -> Path:
    return PKG / f"_host{EXT}"


def device_target() -> Path:
    return PKG / f"_device{EXT}"


def _sources(sub: str, exts: tuple[str, ...]) -> list[Path]:
    return sorted(p for p in (CSRC / sub).rglob("*") if p.suffix in exts)


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


class _Lock:
    def __init__(self, name: str):
        self.path = PKG / f".{name}.buildlock"

    def __enter__(self):
        self.fd = os.open(self.path, os.O_CREAT | os.O_RDWR, 0o644)
        fcntl.flock(self.fd, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        fcntl.flock(self.fd, fcntl.LOCK_UN)
        os.close(self.fd)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print("[ccmpi build]", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"ccmpi build failed: {' '.join(cmd[:3])} ... (exit {r.returncode})")


def build_host(force: bool = False, verbose: bool = False) -> Path:
    srcs = _sources("host", (".cpp",))
    deps = srcs + _sources("host", (".hpp", ".h"))
    target = host_target()
    with _Lock("host"):
        if not force and not _stale(target, deps):
            return target
        cxx = os.environ.get("CXX", "g++")
        with tempfile.TemporaryDirectory() as td:
            tmp = Path(td) / target.name
            cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-Wall",
                   "-Wno-unused-function", *_py_includes(), *map(str, srcs), "-o", str(tmp),
                   "-lrt", "-pthread"]
            _run(cmd, verbose)
            shutil.move(str(tmp), str(target))
    return target


def _torch_lib_dir() -> Path | None:
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            d = Path(spec.origin).parent / "lib"
            return d if d.exists() else None
    except Exception:
        return None
    return None


def build_device(force: bool = False, verbose: bool = False) -> Path:
    """Compile every .hip/.cpp under csrc/device for gfx950 and link `_device`.

    Objects are compiled separately (parallel) then linked with hipcc.  We link
    against /opt/rocm's libamdhip64 / librccl; at run time torch (imported
    first) has already loaded its own copies with the same SONAMEs, so the
    dynamic linker binds our module to those — one HIP runtime per process.
    """
    hip_srcs = _sources("device", (".hip",))
    cpp_srcs = _sources("device", (".cpp",))
    deps = hip_srcs + cpp_srcs + _sources("device", (".hpp", ".h", ".cuh", ".inc"))
    target = device_target()
    with _Lock("device"):
        if not force and not _stale(target, deps):
            return target
        hipcc = str(ROCM / "bin" / "hipcc")
        objdir = PKG / "build" / "device"
        objdir.mkdir(parents=True, exist_ok=True)
        common = ["-O3", "-std=c++20", "-fPIC", "-fvisibility=hidden", f"--offload-arch={ARCH}",
                  f"-I{CSRC / 'device'}", f"-I{ROCM / 'include'}",
                  *_py_includes(), "-Wno-unused-result", "-Wno-unused-command-line-argument"]
        if os.environ.get("CCMPI_SAVE_TEMPS"):
            common += ["-save-temps"]
        objs = []
        procs = []
        for src in hip_srcs + cpp_srcs:
            obj = objdir / (src.stem + ".o")
            objs.append(obj)
            hdrs = _local_includes(src)
            if not force and obj.exists() and not _stale(obj, [src, *hdrs]):
                continue
            cmd = [hipcc, "-x", "hip", *common, "-c", str(src), "-o", str(obj)]
            if verbose:
                print("[ccmpi build]", " ".join(cmd), flush=True)
            procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
            if len(procs) >= int(os.environ.get("MAX_JOBS", "8")):
                _drain(procs)
        _drain(procs)
        with tempfile.TemporaryDirectory() as td:
            tmp = Path(td) / target.name
            cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp),
                   f"-L{ROCM / 'lib'}", "-lamdhip64", "-lrccl", f"-Wl,-rpath,{ROCM / 'lib'}"]
            _run(cmd, verbose)
            _check_own_symbols(tmp)
            shutil.move(str(tmp), str(target))
    return target


def _check_own_symbols(so: Path) -> None:
    """Fail the build when the library references a symbol of our own namespace that
    no object defines (e.g. a kernel template whose host stub hipcc did not emit):
    such a library links, then fails only when it is imported on the GPU box."""
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    r = subprocess.run([nm, "-D", "--undefined-only", str(so)], capture_output=True, text=True)
    missing = [ln.split()[-1] for ln in r.stdout.splitlines() if "_ZN5ccmpi" in ln]
    if missing:
        raise RuntimeError("ccmpi device build: undefined own symbols: " + ", ".join(missing[:8]))


def _local_includes(src: Path) -> list[Path]:
    """Headers a source depends on: its `#include "..."` closure inside csrc/."""
    seen: set[Path] = set()
    todo = [src]
    while todo:
        f = todo.pop()
        for line in f.read_text(errors="ignore").splitlines():
            line = line.strip()
            if line.startswith("#include \""):
                h = (f.parent / line.split('"')[1]).resolve()
                if h.exists() and h not in seen:
                    seen.add(h)
                    todo.append(h)
    return sorted(seen)


def _drain(procs: list) -> None:
    err = None
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out)
            err = f"ccmpi device build failed: {cmd[-3]}"
        elif out and os.environ.get("CCMPI_BUILD_VERBOSE"):
            sys.stderr.write(out)
    procs.clear()
    if err:
        raise RuntimeError(err)


def main(argv: list[str]) -> int:
    what = argv[0] if argv and not argv[0].startswith("-") else "all"
    force = "--force" in argv
    if what in ("host", "all"):
        print(build_host(force=force, verbose=True))
    if what in ("device", "all"):
        print(build_device(force=force, verbose=True))
    return 0


if __name__ == "__main__":
    raise SystemExit(main(sys.argv[1:]))
