"""Build libamphora_hip.so (HIP kernels + C ABI) in-tree for gfx950.

    python tools/build_native.py [--force]     # or __graft_entry__.build()

hipcc cross-compiles without a GPU.  The .so lands next to this file so it
travels with the repo snapshot to the GPU box (it is git-ignored).
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.join(ROOT, "amphora_amd")
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libamphora_hip.so")
SOURCES = [os.path.join(CSRC, f) for f in ("kernels.hip", "wire.hip", "codec.hip", "exchange.hip", "capi.hip")]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in ("field.hpp", "kernels.hpp", "host_stream.hpp", "devio.hpp",
                                                   "b64.hpp", "decimal.hpp")] + [
    os.path.join(ROOT, "include", "amphora.h")]
ARCH = os.environ.get("AMPH_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    return "hipcc"


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def compile_link(out: str, flags, link_flags, objdir: str, verbose: bool = False) -> None:
    """Every translation unit compiled by its own hipcc process at once (the
    fused wire kernels' unit alone takes minutes), then one link.  A unit is
    recompiled when it or a shared header is newer than its object."""
    os.makedirs(objdir, exist_ok=True)
    hdrs = [d for d in DEPS if d not in SOURCES]
    procs = []
    objs = []
    for src in SOURCES:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if os.path.exists(obj) and all(os.path.getmtime(d) <= os.path.getmtime(obj) for d in hdrs + [src]):
            continue
        cmd = [hipcc(), "--offload-arch=%s" % ARCH, "-std=c++17", "-fPIC", "-mcode-object-version=5",
               "-I" + os.path.join(ROOT, "include"), "-c", src, "-o", obj + ".tmp"] + list(flags)
        if verbose:
            print(" ".join(cmd))
        procs.append((obj, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    failed = []
    for obj, p in procs:
        out_text, _ = p.communicate()
        if p.returncode != 0:
            failed.append(obj)
            sys.stderr.write(out_text)
        else:
            os.replace(obj + ".tmp", obj)
    if failed:
        raise RuntimeError("hipcc failed: %s" % ", ".join(os.path.basename(f) for f in failed))
    cmd = [hipcc(), "--offload-arch=%s" % ARCH, "-shared", "-fPIC", "-Wl,-rpath,/opt/rocm/lib", "-o",
           out + ".tmp"] + objs + list(link_flags)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("link failed: %s" % out)
    os.replace(out + ".tmp", out)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    objdir = os.path.join(ROOT, "build", "obj")
    if force:
        for f in os.listdir(objdir) if os.path.isdir(objdir) else []:
            os.remove(os.path.join(objdir, f))
    compile_link(LIB, ["-O3", "-Wall", "-Wno-pass-failed"], [], objdir, verbose)
    return LIB


CPP_TEST_SRC = os.path.join(ROOT, "tests", "cpp", "mirror_test.cpp")
CPP_TEST_BIN = os.path.join(ROOT, "tests", "cpp", "mirror_test")


def build_cpp_test(force: bool = False) -> str:
    """The C++ host-mirror test program (include/amphora.hpp) against the .so."""
    deps = [CPP_TEST_SRC, os.path.join(ROOT, "include", "amphora.hpp"), LIB]
    if not force and os.path.exists(CPP_TEST_BIN) and all(
            os.path.getmtime(d) <= os.path.getmtime(CPP_TEST_BIN) for d in deps):
        return CPP_TEST_BIN
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-I" + os.path.join(ROOT, "include"), CPP_TEST_SRC,
           "-L" + HERE, "-lamphora_hip", "-Wl,-rpath,$ORIGIN/../../amphora_amd", "-o", CPP_TEST_BIN]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("g++ failed building the C++ mirror test")
    return CPP_TEST_BIN


C1_SRC = os.path.join(ROOT, "tools", "c1_native.cpp")
C1_BIN = os.path.join(ROOT, "tools", "c1_native")


def build_c1_native(force: bool = False) -> str:
    """BASELINE config C1 through the C++ mirror (tools/c1_native.cpp)."""
    deps = [C1_SRC, os.path.join(ROOT, "include", "amphora.hpp"), LIB]
    if not force and os.path.exists(C1_BIN) and all(
            os.path.getmtime(d) <= os.path.getmtime(C1_BIN) for d in deps):
        return C1_BIN
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-pthread", "-I" + os.path.join(ROOT, "include"), C1_SRC,
           "-L" + HERE, "-lamphora_hip", "-Wl,-rpath,$ORIGIN/../amphora_amd", "-o", C1_BIN]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("g++ failed building tools/c1_native")
    return C1_BIN


SAN_DIR = os.path.join(ROOT, "build", "sanitize")
SAN_FLAGS = ["-fsanitize=address", "-fsanitize=undefined", "-fno-sanitize-recover=all",
             "-fno-omit-frame-pointer"]


def build_sanitized(force: bool = False) -> dict:
    """Host-code ASan/UBSan builds: the library with its
    host side instrumented (device code untouched -- GPU ASan is not
    available), the C++ mirror test linked against it, and a driver of the C
    oracle.  Output in build/sanitize/ (git-ignored)."""
    os.makedirs(SAN_DIR, exist_ok=True)
    lib = os.path.join(SAN_DIR, "libamphora_hip.so")
    mirror = os.path.join(SAN_DIR, "mirror_test")
    orc = os.path.join(SAN_DIR, "oracle_sanitize")
    orc_src = os.path.join(ROOT, "tests", "cpp", "oracle_sanitize.c")
    if force or not os.path.exists(lib) or any(os.path.getmtime(d) > os.path.getmtime(lib) for d in DEPS):
        san = [x for f in SAN_FLAGS for x in ("-Xarch_host", f)]
        compile_link(lib, ["-O1", "-g"] + san, san, os.path.join(SAN_DIR, "obj"))
    jobs = [
        (mirror, [CPP_TEST_SRC, os.path.join(ROOT, "include", "amphora.hpp"), lib],
         ["/opt/rocm/llvm/bin/clang++", "-std=c++17", "-O1", "-g", "-I" + os.path.join(ROOT, "include"),
          CPP_TEST_SRC, "-L" + SAN_DIR, "-lamphora_hip", "-Wl,-rpath,$ORIGIN", "-o", mirror] + SAN_FLAGS),
        (orc, [orc_src, os.path.join(ROOT, "oracle", "amphora_oracle.c")],
         ["gcc", "-O1", "-g", "-fopenmp", "-Wall", "-Wextra", orc_src, "-o", orc] + SAN_FLAGS),
    ]
    for out, deps, cmd in jobs:
        if not force and os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps):
            continue
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError("sanitizer build failed: %s" % out)
    return {"lib": lib, "mirror": mirror, "oracle": orc}


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_cpp_test(force="--force" in sys.argv))
