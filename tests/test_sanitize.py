"""Sanitizer coverage of the host-side C/C++ (VERDICT r1 missing #7), on the CPU, no GPU:
  * the session host logic (netman_amd/csrc/wsc_session.cpp: pinned staging, carry, prefix
    batches, spills, record-overflow splits, zero-copy views, submit/complete, device-failure
    policy, the cross-thread removal queue) over a host-memory stand-in for the device
    (tests/sanitize/session_stub.cpp), under ASan+UBSan and under TSan with a remover thread;
  * the CPU oracle (oracle/ws_oracle.c) on seeded random and malformed streams under ASan+UBSan.
Every binary exits non-zero on a failed check or any sanitizer report."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "sanitize")
OUT = os.path.join(SAN, "_build")
HIP_INC = ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"]


def _build(name, cmd):
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, name)
    subprocess.run(cmd + ["-o", exe], check=True, capture_output=True, text=True)
    return exe


def _run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1")
    p = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    return p.stdout


SESSION_SRCS = [os.path.join(ROOT, "netman_amd", "csrc", "wsc_session.cpp"), os.path.join(SAN, "session_stub.cpp"),
                os.path.join(SAN, "session_driver.cpp")]


@pytest.mark.parametrize("san,args", [("address,undefined", []), ("thread", ["--threads"])])
def test_session_host_logic_sanitized(san, args):
    exe = _build("session_" + san.split(",")[0],
                 ["g++", "-std=c++17", "-pthread", f"-fsanitize={san}"] + FLAGS + HIP_INC + SESSION_SRCS)
    out = _run(exe, *args)
    assert "0 failed checks" in out


def test_oracle_sanitized():
    exe = _build("oracle_fuzz", ["gcc", "-fsanitize=address,undefined"] + FLAGS +
                 [os.path.join(SAN, "oracle_fuzz.c"), os.path.join(ROOT, "oracle", "ws_oracle.c")])
    assert "runs" in _run(exe)


ECHO_SRCS = [os.path.join(ROOT, "tools", "ws_echo.cpp"), os.path.join(ROOT, "netman_amd", "csrc", "wsc_session.cpp"),
             os.path.join(SAN, "session_stub.cpp")]


@pytest.mark.parametrize("args", [["--pollers", "4"], ["--pollers", "8", "--shutdown"],
                                  ["--pollers", "3", "--frames", "20", "--size", "70000", "--blocking-wait"]])
def test_echo_batcher_thread_sanitized(args):
    """ws_echo --batcher (one batching thread per device owning the session all pollers share:
    feeds and event reads under its lock, the device polled with wsc_session_ready outside it)
    over the host-memory device stand-in, under TSan: real loopback sockets, every echoed byte
    checked by the clients, EOF ordering with --shutdown"""
    exe = _build("ws_echo_batcher_tsan", ["g++", "-std=c++17", "-pthread", "-fsanitize=thread"] + FLAGS + HIP_INC +
                 ECHO_SRCS)
    out = _run(exe, "--batcher", "--conns", "16", "--frames", "50", "--size", "4096", "--client-threads", "2", *args)
    assert '"ok": true' in out
