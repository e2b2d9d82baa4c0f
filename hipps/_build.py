"""In-tree native build for hipps (no hipify, no JIT cache).

Compiles every ``hipps/csrc/**/*.hip`` (device code, gfx950 only) and ``*.cpp`` (host runtime +
pybind11 bindings) with ``hipcc`` and links ``hipps/_C.<abi>.so`` against the torch/HIP/RCCL
libraries that torch itself loads (same sonames, so one HIP runtime and one RCCL per process).

    python -m hipps._build            # incremental
    python -m hipps._build --clean    # full rebuild

``__graft_entry__.build()`` calls :func:`build`.  Sources are compiled in parallel; an object is
rebuilt when its source or any header under csrc/ is newer.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(os.path.dirname(ROOT), "build", "hipps")
ARCH = os.environ.get("HIPPS_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    from torch.utils.cpp_extension import include_paths

    tdir = os.path.dirname(torch.__file__)
    return include_paths(device_type="cuda"), os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(ROOT, "_C" + suffix)


def _sources():
    pats = ["*.hip", "*.cpp", "runtime/*.cpp", "runtime/*.hip"]
    out = []
    for p in pats:
        out += sorted(glob.glob(os.path.join(CSRC, p)))
    return out


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))


def _common_flags(incs, abi):
    py_inc = sysconfig.get_paths()["include"]
    flags = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
             "-DUSE_ROCM=1", "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_C",
             "-DHIP_ENABLE_WARP_SYNC_BUILTINS=1", "-Wno-unused-result", "-Wno-deprecated-declarations"]
    for i in [CSRC, "/opt/rocm/include", py_inc] + list(incs):
        flags.append(f"-I{i}")
    return flags


def _compile(src, obj, flags, verbose):
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    if src.endswith(".hip"):
        cmd = [HIPCC, "-x", "hip", f"--offload-arch={ARCH}", "-fno-gpu-rdc", "-munsafe-fp-atomics"] + flags
    else:
        # host-only translation units still go through hipcc (clang) so HIP runtime headers work
        cmd = [HIPCC] + flags
    cmd += ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return obj


def build(clean: bool = False, verbose: bool = False, jobs: int | None = None) -> str:
    """Compile + link the native extension in-tree; returns the .so path."""
    if clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    incs, tlib, abi = _torch_paths()
    flags = _common_flags(incs, abi)
    srcs = _sources()
    hdr_mtime = max([os.path.getmtime(h) for h in _headers()] + [os.path.getmtime(__file__)])
    todo, objs = [], []
    for s in srcs:
        rel = os.path.relpath(s, CSRC).replace(os.sep, "_")
        o = os.path.join(BUILD, rel + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_mtime):
            todo.append((s, o))
    jobs = jobs or min(8, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(lambda so: _compile(so[0], so[1], flags, verbose), todo))
    out = ext_path()
    if todo or not os.path.exists(out):
        libs = ["-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
                "-lamdhip64", "-lrccl", "-lrocprofiler-sdk-roctx", "-lrt", "-lpthread"]
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out + ".tmp"] + objs + [
            f"-L{tlib}", "-L/opt/rocm/lib", f"-Wl,-rpath,{tlib}"] + libs
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        os.replace(out + ".tmp", out)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    print(build(clean=a.clean, verbose=a.verbose, jobs=a.jobs))


if __name__ == "__main__":
    sys.exit(main())
