"""Build the native library (``python -m myfyp_amd.ops.build``).

Compiles every ``csrc/**/*.hip`` for gfx950 with ``hipcc`` (each translation unit in parallel)
and links ``myfyp_amd/_native/libmyfyp_hip.so`` in-tree, so the ``.so`` travels with the repo
snapshot to the GPU box. Incremental: objects are rebuilt only when a source or header changed.
"""

from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
from typing import List

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
OUT_DIR = os.path.join(ROOT, "myfyp_amd", "_native")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(OUT_DIR, "libmyfyp_hip.so")
HOST_LIB = os.path.join(OUT_DIR, "libmyfyp_host.so")
ARCH = os.environ.get("MYFYP_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-Wno-unused-result"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the native library)")


def sources() -> List[str]:
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.hip"), recursive=True))


def _headers_mtime() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max([os.path.getmtime(h) for h in hs] + [0.0])


def _compile(src: str, hipcc: str, hdr_mtime: float, verbose: bool, obj_dir: str = OBJ_DIR, extra: tuple = ()) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    obj = os.path.join(obj_dir, rel + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime):
        return obj
    cmd = [hipcc, *FLAGS, *extra, "-I", os.path.join(CSRC, "kernels"), "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{res.stdout}\n{res.stderr}")
    return obj


def build(verbose: bool = False, jobs: int = 8, variant: str = "") -> str:
    """Compile + link; returns the library path. ``variant="stamps"`` builds a diagnostic copy with
    per-block phase timestamps (``-DMLP_STAMPS``) under build/stamps/ (select it at run time with
    ``MYFYP_NATIVE_LIB``)."""
    hipcc = _hipcc()
    obj_dir, lib, extra = OBJ_DIR, LIB, ()
    if variant:
        # "stamps" or "stamps+NAME=VAL+NAME2" (extra -D macros for timing-only experiment builds)
        parts = variant.split("+")
        tag = variant.replace("+", "_").replace("=", "").replace("mllvm:", "").replace("-", "")
        obj_dir = os.path.join(ROOT, "build", f"obj_{tag}")
        lib = os.path.join(ROOT, "build", tag, "libmyfyp_hip.so")
        # a part starting with "mllvm:" is a raw backend option (experiment builds: "-mllvm <opt>")
        extra = tuple(["-DMLP_STAMPS"] if parts[0] == "stamps" else [])
        for m in parts[1:]:
            extra += ("-mllvm", m[len("mllvm:"):]) if m.startswith("mllvm:") else (f"-D{m}",)
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    srcs = sources()
    hdr = _headers_mtime()
    with cf.ThreadPoolExecutor(max_workers=min(jobs, max(1, len(srcs)))) as ex:
        objs = list(ex.map(lambda s: _compile(s, hipcc, hdr, verbose, obj_dir, extra), srcs))
    LIB_ = lib
    if not os.path.exists(LIB_) or os.path.getmtime(LIB_) < max(os.path.getmtime(o) for o in objs):
        tmp = LIB_ + ".tmp"
        # the in-process device mesh (csrc/runtime/rccl_mesh.hip) calls RCCL directly; at run time the
        # soname librccl.so.1 resolves to the copy torch already loaded (one RCCL per process)
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp, "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed:\n{res.stdout}\n{res.stderr}")
        os.replace(tmp, LIB_)
    return LIB_


def host_sources() -> List[str]:
    return sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))


def build_host(verbose: bool = False) -> str:
    """Host-only runtime pieces (shared-memory control-plane collectives): plain C++17, built with
    the system compiler so CPU-only hosts have them too. Atomic replace: concurrent ranks may race."""
    srcs = host_sources()
    if os.path.exists(HOST_LIB) and os.path.getmtime(HOST_LIB) >= max(os.path.getmtime(s) for s in srcs):
        return HOST_LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    cxx = os.environ.get("CXX") or shutil.which("g++") or shutil.which("c++") or "/opt/rocm/llvm/bin/clang++"
    tmp = f"{HOST_LIB}.{os.getpid()}.tmp"
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", *srcs, "-o", tmp, "-lrt"]
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"host library build failed:\n{res.stdout}\n{res.stderr}")
    os.replace(tmp, HOST_LIB)
    return HOST_LIB


def build_sanitized(sanitize: str = "thread", verbose: bool = False) -> str:
    """Host runtime + its multi-threaded stress driver (``csrc/host/tests``) built with
    ``-fsanitize=<sanitize>`` ("thread", "address,undefined"): SURVEY §5.2's sanitizer job for the
    native host code. GPU code is not instrumented (no device sanitizers on this pool)."""
    tag = sanitize.replace(",", "_")
    out_dir = os.path.join(ROOT, "build", "sanitize", tag)
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, "shm_collective_stress")
    srcs = host_sources() + sorted(glob.glob(os.path.join(CSRC, "host", "tests", "*.cpp")))
    if os.path.exists(exe) and os.path.getmtime(exe) >= max(os.path.getmtime(s) for s in srcs):
        return exe
    cxx = os.environ.get("CXX") or shutil.which("g++") or "c++"
    cmd = [cxx, "-O1", "-g", "-std=c++17", f"-fsanitize={sanitize}", "-fno-omit-frame-pointer", *srcs, "-o", exe, "-lrt", "-pthread"]
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"sanitizer build failed:\n{res.stdout}\n{res.stderr}")
    return exe


if __name__ == "__main__":
    print(build_host(verbose="-v" in sys.argv))
    print(build(verbose="-v" in sys.argv, variant="stamps" if "--stamps" in sys.argv else ""))
