"""configs[0] loopback echo harness (tools/echo_harness.hpp): every echoed frame is checked byte for
byte by the client threads.  CPU: the reference-port twin (oracle/_build/ws_echo_cpu); GPU: the
product binary tools/ws_echo over libwscodec's wsc_session."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(exe, *args):
    p = subprocess.run([exe, *args], capture_output=True, text=True, timeout=120)
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert line, p.stderr
    return p.returncode, json.loads(line[-1])


@pytest.fixture(scope="module")
def cpu_echo():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return os.path.join(ROOT, "oracle", "_build", "ws_echo_cpu")


@pytest.mark.parametrize("args", [("--conns", "1", "--frames", "50", "--size", "65536"),
                                  ("--conns", "8", "--frames", "40", "--size", "70000", "--client-threads", "2"),
                                  ("--conns", "16", "--frames", "300", "--size", "100", "--client-threads", "4"),
                                  ("--conns", "16", "--frames", "100", "--size", "3000", "--client-threads", "4",
                                   "--pollers", "4")])
def test_cpu_echo_roundtrip(cpu_echo, args):
    rc, d = _run(cpu_echo, *args)
    assert rc == 0 and d["ok"], d
    assert d["messages"] == int(args[1]) * int(args[3])
    # what the server costs its host (round-5 VERDICT #3): poller threads, the whole process minus
    # the client threads, and per GiB echoed
    assert d["poller_cpu_s"] > 0 and d["server_cpu_s"] > 0 and d["client_cpu_s"] > 0, d
    assert d["server_cpu_s"] >= 0.5 * d["poller_cpu_s"], d
    gib = d["messages"] * int(args[5]) / 2**30
    assert abs(d["server_cpu_s_per_gib"] * gib - d["server_cpu_s"]) <= 1e-4 + 0.01 * d["server_cpu_s"], d   # (%.4f)


def test_poller_device_mapping():
    """SURVEY §8(e) / VERDICT r3 #7: ws_echo --devices G puts poller p's session on device p mod G
    (one host thread, stream and pinned staging per GPU; a connection never moves) -- checked
    without a device (--print-map exits before any session is created)"""
    from netman_amd import _build
    exe = _build.build_tools()
    for pollers, devices in ((8, 8), (8, 3), (5, 1), (16, 8)):
        p = subprocess.run([exe, "--pollers", str(pollers), "--conns", "64", "--devices", str(devices), "--print-map"],
                           capture_output=True, text=True, timeout=60)
        d = json.loads(p.stdout)
        assert p.returncode == 0 and d["device_of_poller"] == [i % devices for i in range(pollers)], d


@pytest.mark.parametrize("pollers", ["1", "4"])
def test_cpu_echo_shutdown(cpu_echo, pollers):
    """clients half-close after their last frame: every echo, then the close frame, then FIN"""
    rc, d = _run(cpu_echo, "--conns", "16", "--frames", "40", "--size", "5000", "--client-threads", "4",
                 "--pollers", pollers, "--shutdown")
    assert rc == 0 and d["ok"] and d["shutdown"], d
    assert d["messages"] == 16 * 40


@pytest.mark.gpu
@pytest.mark.parametrize("args", [("--conns", "1", "--frames", "200", "--size", "65536"),
                                  ("--conns", "32", "--frames", "50", "--size", "70000", "--client-threads", "4"),
                                  ("--conns", "16", "--frames", "500", "--size", "125", "--client-threads", "4"),
                                  # 4 pollers x 16 connections, each poller its own
                                  # wsc_session on the one device (eventloop/event.go:33-37)
                                  ("--conns", "64", "--frames", "60", "--size", "65536", "--client-threads", "4",
                                   "--pollers", "4"),
                                  ("--conns", "64", "--frames", "400", "--size", "1024", "--client-threads", "4",
                                   "--pollers", "4", "--sync"),
                                  # one batching thread per device sharing one session among the pollers
                                  ("--conns", "64", "--frames", "60", "--size", "65536", "--client-threads", "4",
                                   "--pollers", "4", "--batcher"),
                                  # blocking-sync completion, reads cut at an odd size (frames split
                                  # across reads and rounds)
                                  ("--conns", "64", "--frames", "60", "--size", "65536", "--client-threads", "4",
                                   "--pollers", "8", "--blocking-wait", "--read-bytes", "100003")])
def test_gpu_echo_roundtrip(codec_lib, args):
    from netman_amd import _build
    exe = _build.build_tools()
    rc, d = _run(exe, *args)
    assert rc == 0 and d["ok"], d
    assert d["messages"] == int(args[1]) * int(args[3])
    assert d["pollers"] == (int(args[args.index("--pollers") + 1]) if "--pollers" in args else 1)
    assert d["server_cpu_s"] > 0 and d["server_cpu_s_per_gib"] > 0, d


@pytest.mark.gpu
@pytest.mark.parametrize("args", [("--pollers", "1"), ("--pollers", "4"), ("--pollers", "4", "--sync"),
                                  ("--pollers", "1", "--conns", "1", "--frames", "300", "--size", "65536")])
def test_gpu_echo_shutdown_delivers_before_close(codec_lib, args):
    """clients send N messages then shutdown(SHUT_WR); the server's read returns 0
    (io.EOF) while messages are still queued or in flight -- every one is echoed, then Close():
    the close frame 88 02 03 E8, then the server's FIN (the client checks all of it)"""
    from netman_amd import _build
    exe = _build.build_tools()
    base = {"--conns": "16", "--frames": "60", "--size": "20000", "--client-threads": "4"}
    a = list(args)
    for k, v in base.items():
        if k not in a:
            a += [k, v]
    rc, d = _run(exe, *a, "--shutdown", "--devices", "1")
    assert rc == 0 and d["ok"] and d["shutdown"], d
    assert d["messages"] == int(a[a.index("--conns") + 1]) * int(a[a.index("--frames") + 1])
    assert d["devices"] == 1
