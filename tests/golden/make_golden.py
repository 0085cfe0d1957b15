"""Generate the committed golden fixtures (run in the build container; aiohttp never travels).

1. rfc6455_kat.json   -- RFC 6455 §5.7 example frames, with the outcome netman's decoder gives them
                         (hand-derived from server/websocket.go / websocket_frame.go; the unmasked
                         examples stall because netman never completes an unmasked header, Q3).
2. aiohttp_streams.bin + aiohttp_expected.json
                      -- seeded valid client streams (masked, fragmented, PING/PONG interleaved,
                         multi-byte UTF-8 split across fragments, 7/16/64-bit lengths) decoded by
                         an independent implementation: aiohttp 3.14.3's pure-Python
                         aiohttp._websocket.reader_py.WebSocketReader.  Expected data messages
                         (opcode, bytes) and PING payloads, in stream order.
Usage: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from netman_amd.synth import frame  # noqa: E402


def kat():
    m = bytes.fromhex("37fa213d")
    cases = [
        dict(name="rfc_single_unmasked_text", hex="810548656c6c6f",
             expect=dict(events=[["STALL"]])),
        dict(name="rfc_single_masked_text", hex="818537fa213d7f9f4d5158",
             expect=dict(events=[["MESSAGE", 0, 1, "48656c6c6f"]])),
        dict(name="rfc_fragmented_unmasked_text", hex="010348656c" + "80026c6f",
             expect=dict(events=[["STALL"]])),
        dict(name="rfc_unmasked_ping", hex="890548656c6c6f", expect=dict(events=[["STALL"]])),
        dict(name="rfc_masked_pong_then_text", hex="8a8537fa213d7f9f4d5158" + "818537fa213d7f9f4d5158",
             expect=dict(events=[["MESSAGE", 1, 1, "48656c6c6f"]])),      # PONG took msgID 0 (Q5)
        dict(name="rfc_256B_unmasked_binary_header", hex="827e0100", pad_zeros=256,
             expect=dict(events=[["STALL"]])),
        dict(name="rfc_64KiB_unmasked_binary_header", hex="827f0000000000010000", pad_zeros=65536,
             expect=dict(events=[["STALL"]])),
        # masked counterparts of the RFC examples (mask 37fa213d)
        dict(name="masked_fragmented_text",
             hex=(frame(1, b"Hel", fin=False, mask=int.from_bytes(m, "little")) +
                  frame(0, b"lo", mask=int.from_bytes(m, "little"))).hex(),
             expect=dict(events=[["MESSAGE", 0, 1, "48656c6c6f"]])),
        dict(name="masked_ping_echo", hex=frame(9, b"Hello", mask=int.from_bytes(m, "little")).hex(),
             expect=dict(events=[["PONG", "48656c6c6f"]])),
        dict(name="masked_256B_binary_16bit_len",
             hex=frame(2, bytes(range(256)), mask=int.from_bytes(m, "little")).hex(),
             expect=dict(events=[["MESSAGE", 0, 2, bytes(range(256)).hex()]])),
        dict(name="masked_64KiB_binary_64bit_len",
             hex=frame(2, b"", mask=int.from_bytes(m, "little")).hex()[:4].replace("8280", "82ff") +
             "0000000000010000" + m.hex(), pad_masked=[0xab, 65536],
             expect=dict(events=[["MESSAGE", 0, 2, "sha256:" + hashlib.sha256(b"\xab" * 65536).hexdigest()]])),
        dict(name="masked_empty_pong_closes", hex=frame(10, b"", mask=1).hex(),
             expect=dict(events=[["CLOSE", 1000, 0]])),
        dict(name="masked_close_1000", hex=frame(8, (1000).to_bytes(2, "big") + b"bye", mask=7).hex(),
             expect=dict(events=[["CLOSE", 1000, 0]])),
        dict(name="masked_close_reserved_1005", hex=frame(8, (1005).to_bytes(2, "big"), mask=7).hex(),
             expect=dict(events=[["CLOSE", 1002, 6]])),
        dict(name="masked_text_bad_utf8", hex=frame(1, b"\xce\xba\xe1\xbd\xb9\xcf\x83\xce\xbc\xce\xb5\xed\xa0\x80", mask=9).hex(),
             expect=dict(events=[["CLOSE", 1007, 5]])),
        dict(name="rsv1_set", hex=frame(2, b"x", rsv=4, mask=3).hex(), expect=dict(events=[["CLOSE", 1002, 2]])),
        dict(name="reserved_opcode_3", hex=frame(3, b"x", mask=3).hex(), expect=dict(events=[["CLOSE", 1002, 1]])),
        dict(name="ping_126_bytes", hex=frame(9, b"p" * 126, mask=3).hex(), expect=dict(events=[["CLOSE", 1002, 3]])),
        dict(name="fragmented_ping", hex=frame(9, b"p", fin=False, mask=3).hex(), expect=dict(events=[["CLOSE", 1002, 4]])),
        dict(name="continuation_without_start", hex=frame(0, b"p", mask=3).hex(), expect=dict(events=[["CLOSE", 1002, 1]])),
    ]
    # Reference quirks and the messageMode-dependent CLOSE rule, each
    # hand-derived from the cited reference lines ("ref").  Not RFC behaviour: netman's.
    T = lambda b, fin=True, m=0x11223344: frame(1, b, fin=fin, mask=m)   # noqa: E731
    B = lambda b, fin=True, m=0x55667788: frame(2, b, fin=fin, mask=m)   # noqa: E731
    cases += [
        dict(name="q5_msgid_counts_ping_and_pong",
             ref="websocket_frame.go:89 (msgID++ for every FIN frame through nextFrame); websocket.go:190,204",
             hex=(frame(9, b"a", mask=1) + frame(10, b"b", mask=2) + B(b"c")).hex(),
             expect=dict(events=[["PONG", "61"], ["MESSAGE", 2, 2, "63"]])),
        dict(name="q6_ping_inside_text_message_valid",
             ref="websocket_frame.go:71 (check keyed on messageMode, not the PING opcode); :84-86 mode kept",
             hex=(T(b"ab", fin=False) + frame(9, b"hi", mask=5) + frame(0, b"c", mask=6)).hex(),
             expect=dict(events=[["PONG", "6869"], ["MESSAGE", 1, 1, "616263"]])),
        dict(name="q6_ping_inside_text_message_invalid",
             ref="websocket_frame.go:71-73 -> WebsocketMustUtf8 -> epoll.go:126-127 CloseCode(1007)",
             hex=(T(b"ab", fin=False) + frame(9, b"\xff", mask=5)).hex(),
             expect=dict(events=[["CLOSE", 1007, 5]])),
        dict(name="q7_fragmented_close_joins_message",
             ref="websocket.go:155-157 (EAGAIN from nextFrame returned); websocket_frame.go:95 continueBuffer += payload",
             hex=(B(b"ab", fin=False) + frame(8, b"\x03\xe8zz", fin=False, mask=2) + frame(0, b"c", mask=3)).hex(),
             expect=dict(events=[["MESSAGE", 0, 2, b"ab\x03\xe8zzc".hex()]])),
        dict(name="q8_empty_fragment_escapes_data_check",
             ref="websocket.go:142-146 (only continueBuffer.Len() >= 1 is rejected)",
             hex=(T(b"", fin=False) + B(b"bin")).hex(),
             expect=dict(events=[["MESSAGE", 0, 2, "62696e"]])),
        dict(name="q8_data_frame_inside_fragmented_message",
             ref="websocket.go:142-146 -> WebsocketPingPayloadOversize -> epoll.go:117-124 CloseCode(1002)",
             hex=(T(b"a", fin=False) + B(b"bin")).hex(),
             expect=dict(events=[["CLOSE", 1002, 3]])),
        dict(name="text_mode_close_whole_invalid_skips_reason",
             ref="websocket.go:155-167: nextFrame's whole-payload utf8.Valid fails (frame.go:71-73), error "
                 "swallowed, stand-in reason DataLen = fragmentLength = 0 after reset() (frame.go:49, "
                 "websocket.go:309) -> :170 skipped; code 1000 valid -> Close() (1000)",
             hex=(T(b"ab", fin=False) + frame(8, b"\x03\xe8\xff", mask=9)).hex(),
             expect=dict(events=[["CLOSE", 1000, 0]])),
        dict(name="text_mode_close_whole_invalid_bad_code",
             ref="as above, then verifyCloseCode(999) (websocket_ctrl.go:162) -> ProtocolError -> 1002",
             hex=(T(b"ab", fin=False) + frame(8, b"\x03\xe7\xff", mask=9)).hex(),
             expect=dict(events=[["CLOSE", 1002, 6]])),
        dict(name="text_mode_close_whole_valid_reason_invalid",
             ref="03 E8 80 80 is valid UTF-8 as a whole, so nextFrame returns the message (Len 4) and "
                 "websocket.go:170 checks payload[2:] = 80 80 -> MustUtf8 -> 1007",
             hex=(T(b"ab", fin=False) + frame(8, b"\x03\xe8\x80\x80", mask=9)).hex(),
             expect=dict(events=[["CLOSE", 1007, 5]])),
        dict(name="bin_mode_close_reason_invalid",
             ref="messageMode BIN: no whole-payload check, websocket.go:170 checks payload[2:] = FF -> 1007",
             hex=(B(b"ab", fin=False) + frame(8, b"\x03\xe8\xff", mask=9)).hex(),
             expect=dict(events=[["CLOSE", 1007, 5]])),
    ]
    return cases


class _Queue:
    """stand-in for aiohttp's WebSocketDataQueue: collects messages"""
    def __init__(self):
        self.msgs = []
        self.exc = None

    def feed_data(self, data, size):
        self.msgs.append(data)

    def set_exception(self, exc, cause=None):
        self.exc = exc

    def feed_eof(self):
        pass


def valid_stream(seed):
    rng = np.random.default_rng(seed)
    out = bytearray()
    texts = ["hello", "Grüße", "日本語", "😀🎉", "ασδφ", "netman ✓"]
    for _ in range(int(rng.integers(5, 30))):
        r = rng.random()
        mk = int(rng.integers(0, 2**32))
        if r < 0.15:
            out += frame(9, bytes(rng.integers(0x20, 0x7F, int(rng.integers(0, 126)), dtype=np.uint8)), mask=mk)
        elif r < 0.5:
            text = rng.random() < 0.5
            if text:
                body = "".join(texts[int(rng.integers(len(texts)))] for _ in range(int(rng.integers(1, 40)))).encode()
            else:
                n = int(rng.choice([0, 5, 125, 126, 1000, 4000] + ([65535, 65536, 70000] if seed % 8 == 0 else [])))
                body = rng.bytes(n)
            k = int(rng.integers(2, 5))
            cuts = sorted(int(x) for x in rng.integers(0, len(body) + 1, k - 1))
            pieces = [body[a:b] for a, b in zip([0] + cuts, cuts + [len(body)])]
            for i, pc in enumerate(pieces):
                op = (1 if text else 2) if i == 0 else 0
                out += frame(op, pc, fin=i == len(pieces) - 1, mask=int(rng.integers(0, 2**32)))
                if i < len(pieces) - 1 and rng.random() < 0.2:
                    out += frame(9, b"mid-ping", mask=int(rng.integers(0, 2**32)))
        else:
            if rng.random() < 0.5:
                body = "".join(texts[int(rng.integers(len(texts)))] for _ in range(int(rng.integers(0, 20)))).encode()
                out += frame(1, body, mask=mk)
            else:
                out += frame(2, rng.bytes(int(rng.choice([0, 1, 124, 125, 126, 127, 300] + ([65536] if seed % 8 == 1 else [])))), mask=mk)
    return bytes(out)


def aiohttp_decode(stream):
    from aiohttp._websocket import reader_py
    from aiohttp.http_websocket import WSMsgType
    q = _Queue()
    rd = reader_py.WebSocketReader(q, max_msg_size=0, compress=False, decode_text=False)
    rd.feed_data(stream)
    assert q.exc is None, q.exc
    out = []
    for m in q.msgs:
        t = m[0] if isinstance(m, tuple) else m.type
        data = m[1] if isinstance(m, tuple) else m.data
        if isinstance(data, str):
            data = data.encode()
        if t == WSMsgType.TEXT:
            out.append(["MESSAGE", 1, data])
        elif t == WSMsgType.BINARY:
            out.append(["MESSAGE", 2, data])
        elif t == WSMsgType.PING:
            out.append(["PONG", None, data])
    return out


def enc(b):
    return b.hex() if len(b) <= 512 else "sha256:" + hashlib.sha256(b).hexdigest() + ":" + str(len(b))


def main():
    with open(os.path.join(HERE, "rfc6455_kat.json"), "w") as f:
        json.dump(kat(), f, indent=1)
    blobs, meta = [], []
    off = 0
    for i in range(40):
        s = valid_stream(0x6A10 + i)
        exp = aiohttp_decode(s)
        meta.append(dict(seed=0x6A10 + i, off=off, len=len(s),
                         expect=[[k, op, enc(d)] for k, op, d in exp]))
        blobs.append(s)
        off += len(s)
    with open(os.path.join(HERE, "aiohttp_streams.bin"), "wb") as f:
        f.write(b"".join(blobs))
    with open(os.path.join(HERE, "aiohttp_expected.json"), "w") as f:
        json.dump(dict(generator="tests/golden/make_golden.py", decoder="aiohttp 3.14.3 reader_py",
                       streams=meta), f, indent=0)
    print("wrote", len(meta), "streams,", off, "bytes")


if __name__ == "__main__":
    main()
