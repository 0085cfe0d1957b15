"""The synthetic generator produces what the oracle decodes as the intended traffic."""
import numpy as np

import oracle_ref as O
from netman_amd import synth


def test_uniform_sizes_and_headers():
    for size, hdr in [(100, 6), (1024, 8), (65535, 8), (65536, 14)]:
        cfg = synth.uniform_batch(8, size, 4, seed=1)
        assert len(cfg["wire"]) == 8 * (size + hdr)
        ev = O.run(bytes(cfg["wire"][:int(cfg["seg_off"][1])])).events
        assert [e.msg_id for e in ev] == [0, 1, 2, 3] and all(len(e.data) == size for e in ev)
        ref = synth.unmask_reference(cfg["wire"], cfg["payload_off"], cfg["plen"], cfg["mask"])
        p = int(cfg["payload_off"][0])
        assert ref[p:p + size].tobytes() == ev[0].data


def test_fragmented_batch_one_message_per_connection():
    cfg = synth.fragmented_batch(n_conns=50, seed=3, ping_p=0.2)
    for i in range(50):
        a, b = int(cfg["seg_off"][i]), int(cfg["seg_off"][i + 1])
        ev = O.run(bytes(cfg["wire"][a:b])).events
        msgs = [e for e in ev if e.type == O.EV_MESSAGE]
        assert len(msgs) == 1 and msgs[0].opcode == 2
        assert all(e.type in (O.EV_MESSAGE, O.EV_PONG) for e in ev)


def test_mixed_batch_distribution():
    cfg = synth.mixed_batch(n_frames=20000, seed=synth.SEED_BASE + 2)
    u, c = np.unique(cfg["plen"], return_counts=True)
    assert set(u.tolist()) <= {125, 65536, 1048576}
    assert c[0] > 19000
