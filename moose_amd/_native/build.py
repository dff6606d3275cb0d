"""Build the native core ``libmoosex.so`` in-tree.

Host sources (``csrc/*.cpp``) are compiled with g++ (AES-NI, ``unsigned __int128``);
device sources (``csrc/*.hip``) with ``hipcc --offload-arch=gfx950``.  The shared
library lands next to this file so that it travels with the repository snapshot to a
GPU box.  Objects are rebuilt only when a source or header is newer than the object.
"""
from __future__ import annotations

import fcntl
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
CSRC = REPO / "csrc"
BUILD = REPO / "build" / "native"
LIB = HERE / "libmoosex.so"
ARCH = os.environ.get("MOOSEX_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


def _sources():
    return sorted(CSRC.glob("*.cpp")) + sorted(CSRC.glob("*.hip"))


def _headers_mtime():
    hs = list(CSRC.glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


# Per-source extra flags.  gemm_crt.hip: let the MFMA accumulators live in VGPRs and the
# allocator use the AGPR half of the unified register file for the rest, so the 4-wave
# 128x128 wave-tile variants (256 accumulators per lane, one wave per SIMD) compile without
# scratch spills (default form: 275 spilled VGPRs).  The 8-wave variants' code is unchanged.
_HIP_EXTRA = {"gemm_crt.hip": ("-mllvm", "-amdgpu-mfma-vgpr-form=1")}


def _compile(src: Path, obj: Path, verbose: bool):
    if src.suffix == ".hip":
        cmd = [
            HIPCC,
            f"--offload-arch={ARCH}",
            "-O3",
            "-fPIC",
            "-std=c++17",
            "-Wno-unused-result",
            *_HIP_EXTRA.get(src.name, ()),
            "-c",
            str(src),
            "-o",
            str(obj),
        ]
    else:
        cmd = [
            CXX,
            "-O3",
            "-fPIC",
            "-std=c++17",
            "-pthread",
            "-msse4.1",
            "-c",
            str(src),
            "-o",
            str(obj),
        ]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src.name}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = False) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    lock_path = BUILD / ".lock"
    with open(lock_path, "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        hdr = _headers_mtime()
        jobs = []
        objs = []
        for src in _sources():
            obj = BUILD / (src.name + ".o")
            objs.append(obj)
            stale = (
                force
                or not obj.exists()
                or obj.stat().st_mtime < max(src.stat().st_mtime, hdr)
            )
            if stale:
                jobs.append((src, obj))
        if jobs:
            with ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
                list(ex.map(lambda j: _compile(j[0], j[1], verbose), jobs))
        newest_obj = max(o.stat().st_mtime for o in objs)
        if force or jobs or not LIB.exists() or LIB.stat().st_mtime < newest_obj:
            tmp = LIB.with_suffix(".so.tmp")
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread"]
            cmd += [str(o) for o in objs] + ["-o", str(tmp)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
            os.replace(tmp, LIB)
        return LIB


def needs_build() -> bool:
    if not LIB.exists():
        return True
    lib_t = LIB.stat().st_mtime
    newest = max([s.stat().st_mtime for s in _sources()] + [_headers_mtime()])
    return newest > lib_t


RT_SRC = CSRC / "runtime"
RT_EXT = HERE / ("_moosert" + sysconfig.get_config_var("EXT_SUFFIX"))


def runtime_needs_build() -> bool:
    srcs = list(RT_SRC.glob("*.cpp")) + list(RT_SRC.glob("*.h"))
    if not RT_EXT.exists():
        return True
    return bool(srcs) and max(p.stat().st_mtime for p in srcs) > RT_EXT.stat().st_mtime


def build_runtime(force: bool = False, verbose: bool = False) -> Path:
    """Native runtime core (csrc/runtime: parser, graph passes, TCP networking, dataflow
    scheduler, pybind11 bindings) -> moose_amd/_native/_moosert*.so (host C++)."""
    import pybind11

    BUILD.mkdir(parents=True, exist_ok=True)
    with open(BUILD / ".lock_rt", "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        if not force and not runtime_needs_build():
            return RT_EXT
        tmp = RT_EXT.with_name(RT_EXT.name + ".tmp")
        cmd = [CXX, "-O2", "-fPIC", "-std=c++17", "-pthread", "-shared",
               "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]
        cmd += [str(s) for s in sorted(RT_SRC.glob("*.cpp"))] + ["-o", str(tmp)]
        cmd += ["-lssl", "-lcrypto"]  # mutual TLS of the TCP networking
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"runtime build failed\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, RT_EXT)
    return RT_EXT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_runtime(force="--force" in sys.argv, verbose=True))
