"""The byte source with TLS on (VERDICT r4 "next" #1, row (b)/A10).

With TLS on, BaseConnect.readData reads through tls.Conn.Read (server/baseconnect.go:347-353; the
layer is built at :56-63, the poller finishes the TLS handshake before DecodePacket,
eventloop/epoll.go:85-102).  A tls.Conn returns at most one record's plaintext per Read and keeps
the records it has already pulled off the socket in its own buffers, where level-triggered epoll
cannot see them.  INTEGRATION.md's Session.ReadTLS therefore reads into the reserved staging until
the layer reports EAGAIN (or the room is full: `more`, read again next round) and maps the layer's
io.EOF to wsc_session_eof.  codec.Session.read_tls is the same loop; FakeTLSConn stands in for the
tls.Conn (Go is absent here and on the box).  Expected events: O.run on the whole plaintext stream.
"""
from collections import deque

import numpy as np
import pytest

import oracle_ref as O
from fuzz_streams import random_stream
from gpu_helpers import events_of_session
from netman_amd import codec as K
from netman_amd import synth

pytestmark = pytest.mark.gpu

RECORD = 16384        # TLS max plaintext per record (RFC 8446 5.1)


class FakeTLSConn:
    """tls.Conn over a non-blocking socket.  Records arrive on the 'socket'; read(n) first pulls
    every record the socket holds into the layer (the socket is then empty, so EPOLLIN stops
    firing) and returns up to n bytes of ONE record; EAGAIN (BlockingIOError) when nothing is
    buffered; b"" (io.EOF) once the peer's FIN has arrived and everything was read."""

    def __init__(self, plaintext: bytes, rng, fin: bool):
        self.pending = deque()
        i = 0
        while i < len(plaintext):
            k = int(rng.integers(1, RECORD + 1))
            self.pending.append(plaintext[i:i + k])
            i += k
        self.fin = fin
        self.socket, self.buffered = deque(), deque()
        self.cur = b""
        self.fin_arrived = False

    def arrive(self, k: int):
        for _ in range(min(k, len(self.pending))):
            self.socket.append(self.pending.popleft())
        if not self.pending and self.fin:
            self.fin_arrived = True

    def epollin(self) -> bool:           # level-triggered: bytes or the FIN on the socket
        return bool(self.socket) or self.fin_arrived

    def read(self, n: int) -> bytes:
        self.buffered.extend(self.socket)
        self.socket.clear()
        if not self.cur:
            if self.buffered:
                self.cur = self.buffered.popleft()
            elif self.fin_arrived:
                return b""
            else:
                raise BlockingIOError
        out, self.cur = self.cur[:n], self.cur[n:]
        return out

    def drained(self) -> bool:
        return not (self.pending or self.socket or self.buffered or self.cur)


def _poll(sess, conns, layers, rng, max_read, loop_reads, pipelined, max_rounds=4000):
    """the poller of INTEGRATION.md (2): a connection is read when EPOLLIN fires, or when its last
    ReadTLS filled the room (more) or its websocket handshake just finished (first round)"""
    got = {c: [] for c in conns}
    more = {c: True for c in conns}          # set by the handshake branch of DecodePacket
    done = {c: False for c in conns}         # read side finished: io.EOF read, or the connection closed

    def closed(c):                           # Close()/CloseCode or Q3 stall delivered: the shim stops reading
        return any(e[0] in (K.EV_CLOSE, K.EV_STALL) for e in got[c])

    def finished(c, L):
        return closed(c) or (L.drained() and not more[c] and (done[c] or not L.fin))

    for r in range(max_rounds):
        for c, L in zip(conns, layers):
            L.arrive(int(rng.integers(0, 4)))
        for c, L in zip(conns, layers):
            if done[c] or closed(c) or not (L.epollin() or more[c]):
                continue
            if loop_reads:
                n, more[c], eof = sess.read_tls(c, L, max_read)
            else:                            # one tls.Conn.Read per readiness event (wrong)
                more[c] = False
                try:
                    b = L.read(max_read)
                    eof = not b
                    if b:
                        sess.feed(c, b)
                except BlockingIOError:
                    eof = False
            if eof:
                sess.eof(c)
                done[c] = True
        if pipelined:
            sess.submit()
            for c in conns:
                got[c].extend(events_of_session(sess, c))
            sess.complete()
        else:
            sess.decode()
        for c in conns:
            got[c].extend(events_of_session(sess, c))
        if all(finished(c, L) for c, L in zip(conns, layers)) and sess.pending() == 0:
            if pipelined:
                sess.submit()
                sess.complete()
                for c in conns:
                    got[c].extend(events_of_session(sess, c))
            return got, r
    return got, None


def _streams(seed):
    rng = np.random.default_rng(seed)
    s = [random_stream(seed + i, n_units=20, pong_big_p=0.05) for i in range(10)]
    s.append(synth.frame(2, rng.bytes(300_000), mask=5) + synth.frame(1, "✓ done".encode(), mask=6))
    s.append(b"".join(synth.frame(2, rng.bytes(int(rng.integers(0, 3000))), mask=int(rng.integers(1, 1 << 32)))
                      for _ in range(200)))
    return s


@pytest.mark.parametrize("max_read,pipelined", [(4 << 20, False), (RECORD, False), (5000, True)])
def test_tls_reads_drain_the_record_layer(codec_lib, max_read, pipelined):
    """wss: the shim's ReadTLS loop delivers exactly O.run(stream, eof=True) for every connection,
    however the records arrive; a room smaller than the buffered plaintext (5,000 B, one record)
    is continued through `more` without any EPOLLIN"""
    rng = np.random.default_rng(5)
    streams = _streams(4100)
    sess = K.Session(0, max_batch_bytes=1 << 20, max_segs=64, max_frames=1 << 14)
    conns = [sess.open() for _ in streams]
    layers = [FakeTLSConn(s, rng, fin=True) for s in streams]
    got, rounds = _poll(sess, conns, layers, rng, max_read, loop_reads=True, pipelined=pipelined)
    assert rounds is not None, "the poller did not drain"
    for i, (c, s) in enumerate(zip(conns, streams)):
        assert got[c] == [e.key() for e in O.run(s, cap=1 << 12, eof=True).events], f"stream {i}"
    sess.close()


def test_tls_single_read_per_epollin_strands_plaintext(codec_lib):
    """why the loop: with one tls.Conn.Read per readiness event and a client that keeps the
    connection open (no FIN), records the layer already pulled off the socket are never read --
    epoll does not fire for them -- while the ReadTLS loop delivers every message"""
    rng = np.random.default_rng(9)
    streams = _streams(4200)
    results = {}
    for loop in (False, True):
        sess = K.Session(0, max_batch_bytes=1 << 20, max_segs=64, max_frames=1 << 14)
        conns = [sess.open() for _ in streams]
        layers = [FakeTLSConn(s, np.random.default_rng(1), fin=False) for s in streams]
        got, _ = _poll(sess, conns, layers, np.random.default_rng(2), 4 << 20, loop_reads=loop,
                       pipelined=False, max_rounds=400)
        results[loop] = (got, conns, layers)
        sess.close()
    got, conns, layers = results[True]
    for c, s, L in zip(conns, streams, layers):
        assert L.drained() or any(e[0] in (K.EV_CLOSE, K.EV_STALL) for e in got[c])
        assert got[c] == [e.key() for e in O.run(s, cap=1 << 12).events]
    got, conns, layers = results[False]
    assert not all(L.drained() for L in layers)
    assert sum(len(got[c]) for c in conns) < sum(len(results[True][0][c]) for c in results[True][1])
