"""Loading the committed golden fixtures (tests/golden/)."""
import hashlib
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def kat_cases():
    cases = json.load(open(os.path.join(GOLDEN, "rfc6455_kat.json")))
    out = []
    for c in cases:
        b = bytearray(bytes.fromhex(c["hex"]))
        if "pad_zeros" in c:
            b += bytes(c["pad_zeros"])
        if "pad_masked" in c:
            val, n = c["pad_masked"]
            m = b[-4:]
            b += bytes(val ^ m[i % 4] for i in range(n))
        out.append((c["name"], bytes(b), c["expect"]["events"]))
    return out


def aiohttp_cases():
    meta = json.load(open(os.path.join(GOLDEN, "aiohttp_expected.json")))
    blob = open(os.path.join(GOLDEN, "aiohttp_streams.bin"), "rb").read()
    return [(m["seed"], blob[m["off"]:m["off"] + m["len"]], m["expect"]) for m in meta["streams"]]


def data_matches(enc: str, data: bytes) -> bool:
    if enc.startswith("sha256:"):
        parts = enc.split(":")
        ok = hashlib.sha256(data).hexdigest() == parts[1]
        return ok and (len(parts) < 3 or int(parts[2]) == len(data))
    return bytes.fromhex(enc) == data


def event_matches(exp, ev) -> bool:
    """exp: ["MESSAGE", msg_id, opcode, data] | ["PONG", data] | ["CLOSE", code, err] | ["STALL"]"""
    from oracle_ref import EV_MESSAGE, EV_PONG, EV_CLOSE, EV_STALL
    k = exp[0]
    if k == "MESSAGE":
        return ev.type == EV_MESSAGE and ev.msg_id == exp[1] and ev.opcode == exp[2] and data_matches(exp[3], ev.data)
    if k == "PONG":
        return ev.type == EV_PONG and data_matches(exp[1], ev.data)
    if k == "CLOSE":
        return ev.type == EV_CLOSE and ev.close_code == exp[1] and ev.err == exp[2]
    if k == "STALL":
        return ev.type == EV_STALL
    return False
