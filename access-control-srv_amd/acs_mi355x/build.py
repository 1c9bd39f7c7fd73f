"""Build the native libraries in-tree (hipcc, gfx950).

  lib/libacs_mi355x.so          product: HIP kernels + C ABI (include/acs_mi355x.h)
  lib/acs_mi355x.node           N-API addon over the C ABI for a Node/TS host (gcc; needs
                                /usr/include/node, skipped when the headers are absent)
  tests/native/libacs_core_host.so   test infrastructure: the evaluator core on the CPU

Both are plain ``hipcc -shared`` builds so the .so files travel with the repo
snapshot to the GPU box (no JIT cache).  Rebuilds only when a source is newer.
"""
from __future__ import annotations

import os
import subprocess

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib", "libacs_mi355x.so")
HOST_LIB = os.path.join(ROOT, "tests", "native", "libacs_core_host.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# host code (codec, compiler, validation): x86-64-v3 (AVX2 / BMI2 / POPCNT), which every EPYC host
# of an MI355X and this build container have; ACS_HOST_ARCH="" builds baseline x86-64
HOST_ARCH = [f"-march={a}" for a in [os.environ.get("ACS_HOST_ARCH", "x86-64-v3")] if a]

_HEADERS = [os.path.join(CSRC, f) for f in ("acs_layout.h", "acs_eval.h", "acs_json.h", "acs_pool.h")] + \
    [os.path.join(ROOT, "include", "acs_mi355x.h")]
# host-only C++ of the product library: the native request codec and its JSON reader
_HOST_SRCS = [os.path.join(CSRC, f) for f in ("acs_codec.cpp", "acs_compiler.cpp", "acs_json.cpp", "acs_validate.cpp")]


def _stale(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def _hipcc(src, out, extra=(), host_srcs=()):
    """hipcc for gfx950; `host_srcs` (plain C++, no device code) are compiled with g++ into
    objects next to `out` and linked into the same shared library."""
    os.makedirs(os.path.dirname(out), exist_ok=True)
    objs = []
    for h in host_srcs:
        o = out + "." + os.path.basename(h) + ".o"
        subprocess.run(["g++", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-pthread", *HOST_ARCH,
                        "-I", CSRC, "-I", os.path.join(ROOT, "include"), *extra, "-c", h, "-o", o], check=True)
        objs.append(o)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-Wno-unused-function", "-I", CSRC, "-I", os.path.join(ROOT, "include"), *extra, src,
           *(["-x", "none", *objs] if objs else []),
           "-lpthread", "-o", out + ".tmp"]
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    for o in objs:
        os.remove(o)


def build_product(force=False):
    src = os.path.join(CSRC, "acs_kernels.hip")
    if force or _stale(LIB, [src] + _HEADERS + _HOST_SRCS):
        _hipcc(src, LIB, host_srcs=_HOST_SRCS)
    return LIB


PROF_LIB = os.path.join(PKG, "lib", "libacs_mi355x_prof.so")


def build_prof(force=False):
    """Phase-profiling variant of the product library (-DACS_PHASE_PROF; tools/phase_prof.py)."""
    src = os.path.join(CSRC, "acs_kernels.hip")
    if force or _stale(PROF_LIB, [src] + _HEADERS + _HOST_SRCS):
        _hipcc(src, PROF_LIB, ("-DACS_PHASE_PROF",), host_srcs=_HOST_SRCS)
    return PROF_LIB


SCAN_LIB = os.path.join(PKG, "lib", "libacs_mi355x_scan.so")


def build_scan(force=False):
    """Counting variant of the product library (-DACS_SCAN_COUNT): every table read a wave
    issues adds its bytes to a device counter (bench.py's measured B_scan)."""
    src = os.path.join(CSRC, "acs_kernels.hip")
    if force or _stale(SCAN_LIB, [src] + _HEADERS + _HOST_SRCS):
        _hipcc(src, SCAN_LIB, ("-DACS_SCAN_COUNT",), host_srcs=_HOST_SRCS)
    return SCAN_LIB


def build_variant(name, defines, force=False):
    """Experimental build of the product library with extra -D flags (lib/variants/<name>.so)."""
    out = os.path.join(PKG, "lib", "variants", name + ".so")
    src = os.path.join(CSRC, "acs_kernels.hip")
    if force or _stale(out, [src] + _HEADERS + _HOST_SRCS):
        _hipcc(src, out, tuple("-D" + d for d in defines), host_srcs=_HOST_SRCS)
    return out


NAPI_SRC = os.path.join(PKG, "napi", "acs_napi.c")
NAPI_OUT = os.path.join(PKG, "lib", "acs_mi355x.node")
NODE_INC = "/usr/include/node"


def build_napi(force=False):
    """gcc build of the N-API addon, linked to libacs_mi355x.so via $ORIGIN (None if no headers)."""
    if not os.path.exists(os.path.join(NODE_INC, "node_api.h")):
        return None
    lib = build_product()
    if force or _stale(NAPI_OUT, [NAPI_SRC, lib, os.path.join(ROOT, "include", "acs_mi355x.h")]):
        cmd = ["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-pthread", "-Wall", "-Wextra", "-Wno-unused-parameter",
               "-I", NODE_INC, NAPI_SRC, "-o", NAPI_OUT + ".tmp", "-L", os.path.dirname(lib), "-lacs_mi355x",
               "-Wl,-rpath,$ORIGIN"]
        subprocess.run(cmd, check=True)
        os.replace(NAPI_OUT + ".tmp", NAPI_OUT)
    return NAPI_OUT


def build_host_core(force=False):
    src = os.path.join(ROOT, "tests", "native", "core_host.hip")
    if force or _stale(HOST_LIB, [src] + _HEADERS):
        _hipcc(src, HOST_LIB)
    return HOST_LIB


def build_all(force=False):
    """The product, the counting build and the host core compile in parallel (each hipcc run is
    single-threaded and takes minutes); the addon links against the product afterwards."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(3) as ex:
        jobs = [ex.submit(f, force) for f in (build_product, build_host_core, build_scan)]
        lib, host, scan = [j.result() for j in jobs]
    return lib, host, build_napi(force), scan


if __name__ == "__main__":
    print(build_all(force=True))
