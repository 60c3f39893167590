"""In-tree native build: the C++ scheduling core (g++) and the HIP/CDNA4 kernels (hipcc).

Everything is compiled with explicit compiler command lines (no hipify, no JIT cache
under ~/.cache) so the produced ``.so`` files live inside the package directory and
travel with the repository snapshot to the GPU box.

* ``_dlsched_core*.so`` — csrc/core + csrc/runtime, pure C++17 + pybind11.
* ``_dlsched_ops*.so``  — csrc/kernels/*.hip compiled for ``--offload-arch=gfx950``
  plus a torch binding translation unit; it links against torch's bundled
  ``libamdhip64.so.7`` (same soname as /opt/rocm's, resolved to the already-loaded one).
"""
from __future__ import annotations

import glob
import hashlib
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD_DIR = os.path.join(REPO, "build", "native")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("DLS_OFFLOAD_ARCH", "gfx950")

CORE_SO = os.path.join(PKG_DIR, "_dlsched_core" + EXT)
OPS_SO = os.path.join(PKG_DIR, "_dlsched_ops" + EXT)


def _newer(out: str, srcs) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def _digest(srcs) -> str:
    h = hashlib.sha256()
    for s in sorted(srcs):
        h.update(os.path.relpath(s, REPO).encode())
        with open(s, "rb") as f:
            h.update(f.read())
    h.update(ARCH.encode())
    return h.hexdigest()


def _stale(out: str, srcs) -> bool:
    """Does the library need a rebuild? By the sources' CONTENT hash recorded next to it at
    link time (a copied snapshot — the GPU box, a fresh clone — keeps no meaningful mtimes,
    and a rebuild there would be minutes of hipcc per process); by mtimes only when no
    record exists."""
    if not os.path.exists(out):
        return True
    stamp = out + ".srchash"
    if os.path.exists(stamp):
        with open(stamp) as f:
            return f.read().strip() != _digest(srcs)
    return _newer(out, srcs)


def _record(out: str, srcs, digest: str = None) -> None:
    """Stamp ``out`` with the sources' digest — taken BEFORE the compile started (``digest``),
    so a source edited while the compiler ran leaves the output stale, not falsely fresh."""
    with open(out + ".srchash.tmp", "w") as f:
        f.write(digest or _digest(srcs))
    os.replace(out + ".srchash.tmp", out + ".srchash")


class _BuildLock:
    """Cross-process lock around a staleness check + build: the ranks of a multi-GPU job import
    the package at the same time, and only one of them may compile (the others wait, then find
    the library fresh)."""

    def __init__(self, name: str):
        os.makedirs(BUILD_DIR, exist_ok=True)
        self.path = os.path.join(BUILD_DIR, name + ".lock")
        self.f = None

    def __enter__(self):
        import fcntl

        self.f = open(self.path, "a+")
        fcntl.flock(self.f.fileno(), fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl

        fcntl.flock(self.f.fileno(), fcntl.LOCK_UN)
        self.f.close()


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build_core(force: bool = False, verbose: bool = False) -> str:
    import pybind11

    srcs = sorted(glob.glob(os.path.join(CSRC, "core", "*.cpp")) + glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "core", "*.h")) + glob.glob(os.path.join(CSRC, "runtime", "*.h")))
    if not force and not _stale(CORE_SO, srcs + hdrs):
        return CORE_SO
    with _BuildLock("core"):
        if not force and not _stale(CORE_SO, srcs + hdrs):
            return CORE_SO  # another process built it while we waited
        return _build_core(srcs, hdrs, pybind11, verbose)


def _build_core(srcs, hdrs, pybind11, verbose) -> str:
    d0 = _digest(srcs + hdrs)
    cmd = [
        os.environ.get("CXX", "g++"), "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
        "-Wall", "-Wno-sign-compare",
        f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
        *srcs, "-o", CORE_SO + ".tmp",
    ]
    _run(cmd, verbose)
    os.replace(CORE_SO + ".tmp", CORE_SO)
    _record(CORE_SO, srcs + hdrs, d0)
    return CORE_SO


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce

    inc = [f"-I{p}" for p in ce.include_paths()] + [f"-I{sysconfig.get_paths()['include']}"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_dlsched_ops",
            "-DTORCH_API_INCLUDE_EXTENSION_H", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1"]
    libdir = ce.library_paths()[0]
    libs = [f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
            "-lc10_hip", "-ltorch_hip", "-lamdhip64"]
    return inc, defs, libs


def build_ops(force: bool = False, verbose: bool = False, jobs: int = 8) -> str:
    """Compile every csrc/kernels/*.hip for gfx950 and link the torch op library."""
    kern = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    # host C++ against torch: the op bindings, the native step runner (runner.cpp) and the
    # loopback hub; their own headers (*.hpp, csrc/runtime/p2p_match.h) are host-only, so editing
    # them does not recompile the kernels
    hosts = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.cpp")))
    host_hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hpp"))) + [os.path.join(CSRC, "runtime", "p2p_match.h")]
    srcs = kern + hdrs + hosts + host_hdrs
    if not force and not _stale(OPS_SO, srcs):
        return OPS_SO
    with _BuildLock("ops"):
        if not force and not _stale(OPS_SO, srcs):
            return OPS_SO  # another process built it while we waited
        return _build_ops(kern, hdrs, hosts, host_hdrs, force, verbose, jobs)


def _build_ops(kern, hdrs, hosts, host_hdrs, force, verbose, jobs) -> str:
    os.makedirs(BUILD_DIR, exist_ok=True)
    d0 = _digest(kern + hdrs + hosts + host_hdrs)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    inc, defs, libs = _torch_flags()
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
              f"-I{os.path.join(CSRC, 'kernels')}"]

    # per-file code-generation options: the attention kernel's accumulators feed VALU softmax
    # math every tile, so it takes the VGPR form of the MFMAs (no accvgpr read/write shuffles);
    # the GEMMs keep the default (their accumulators only meet the VALU in the epilogue)
    per_file = {"attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}

    def compile_kernel(src):
        # objects are stamped by content too (an mtime check misses an edit made while an
        # earlier compile of the same file was running)
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        if force or _stale(obj, [src] + hdrs):
            d = _digest([src] + hdrs)
            _run([hipcc, *common, *per_file.get(os.path.basename(src), []), "-c", src, "-o", obj], verbose)
            _record(obj, [src] + hdrs, d)
        return obj

    def compile_host(src):
        obj = os.path.join(BUILD_DIR, os.path.splitext(os.path.basename(src))[0] + ".o")
        deps = [src] + hdrs + host_hdrs
        if force or _stale(obj, deps):
            d = _digest(deps)
            _run([hipcc, "-O2", "-std=c++17", "-fPIC", *inc, *defs, f"-I{os.path.join(CSRC, 'kernels')}",
                  f"-I{ROCM}/include", "-x", "c++", "-c", src, "-o", obj], verbose)
            _record(obj, deps, d)
        return obj

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(compile_kernel, kern)) + list(ex.map(compile_host, hosts))
    _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, *libs, "-o", OPS_SO + ".tmp"], verbose)
    os.replace(OPS_SO + ".tmp", OPS_SO)
    _record(OPS_SO, kern + hdrs + hosts + host_hdrs, d0)
    return OPS_SO


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_core(force=force, verbose=verbose)
    if glob.glob(os.path.join(CSRC, "kernels", "*.hip")):
        build_ops(force=force, verbose=verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, verbose=True)
