"""Build recipes for the in-tree native libraries (gfx950 only).

libwscodec.so  <- netman_amd/csrc/{wsc_kernels.hip, wsc_unmask_{inplace,compact}.hip, wsc_encode.hip,
                  wsc_api.cpp, wsc_session.cpp}   (hipcc, translation units compiled in parallel)
The oracle (test infrastructure) has its own recipe in oracle/Makefile; __graft_entry__.build()
drives both.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libwscodec.so")
SOURCES = ["wsc_kernels.hip", "wsc_unmask_inplace.hip", "wsc_unmask_compact.hip", "wsc_encode.hip",
           "wsc_api.cpp", "wsc_session.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def _newest(paths):
    return max(os.path.getmtime(p) for p in paths)


def build_codec(force=False, verbose=False):
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, "wsc_kernels.hpp"), os.path.join(CSRC, "wsc_dev.hpp"),
                   os.path.join(CSRC, "wsc_unmask.inl"),
                   os.path.join(CSRC, "wsc_u8.hpp"), os.path.join(CSRC, "wsc_u8check.inl"),
                   os.path.join(ROOT, "include", "wscodec.h")]
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _newest(deps):
        return LIB
    objs, procs = [], []
    for s in srcs:   # compile the translation units in parallel
        o = os.path.join("/tmp", "wsc_" + os.path.basename(s) + ".o")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
               "-x", "hip", "-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd))
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(o)
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    tmp = LIB + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


TOOLS = os.path.join(ROOT, "tools")
ECHO = os.path.join(TOOLS, "ws_echo")


def build_tools(force=False):
    """tools/ws_echo (configs[0] loopback echo through libwscodec's wsc_session); needs the library"""
    src = os.path.join(TOOLS, "ws_echo.cpp")
    deps = [src, os.path.join(TOOLS, "echo_harness.hpp"), os.path.join(ROOT, "include", "wscodec.h"), LIB]
    if not force and os.path.exists(ECHO) and os.path.getmtime(ECHO) >= _newest(deps):
        return ECHO
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-pthread", "-o", ECHO, src, "-L" + HERE, "-lwscodec",
           "-Wl,-rpath,$ORIGIN/../netman_amd", "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True)
    return ECHO


def build_oracle(force=False):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")] + (["-B"] if force else []),
                   check=True)
