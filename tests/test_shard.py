"""Sharding logic on CPU, incl. a world_size-2 gloo run of the N>1 path (barrier + max-over-ranks,
independent per-rank shards decoded by the oracle)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from netman_amd import shard, synth


def test_split_batch_roundtrip():
    cfg = synth.uniform_batch(64, 300, 3, seed=5)
    parts = [shard.split_batch(cfg["wire"], cfg["seg_off"], 4, r) for r in range(4)]
    assert sum(len(p[2]) for p in parts) == len(cfg["seg_off"]) - 1
    for r, (w, off, mine) in enumerate(parts):
        assert (mine % 4 == r).all()
        for j, s in enumerate(mine):
            a, b = int(cfg["seg_off"][s]), int(cfg["seg_off"][s + 1])
            assert np.array_equal(w[int(off[j]):int(off[j + 1])], cfg["wire"][a:b])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    import oracle_ref as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = synth.uniform_batch(32, 1000, 4, seed=shard.shard_seed(synth.SEED_BASE, rank))
    dist.barrier()
    evs = 0
    for i in range(len(cfg["seg_off"]) - 1):
        a, b = int(cfg["seg_off"][i]), int(cfg["seg_off"][i + 1])
        evs += len(O.run(bytes(cfg["wire"][a:b])).events)
    t = shard.max_over_ranks(float(rank + 1), dist)
    q.put((rank, evs, t, int(cfg["mask"][0])))
    dist.destroy_process_group()


def test_gloo_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [32, 32]          # every frame of every shard delivered
    assert [r[2] for r in res] == [2.0, 2.0]        # max over ranks
    assert res[0][3] != res[1][3]                   # independent shards
    assert abs(shard.aggregate_rate([2**30, 2**30], 1.0, 1) - 2.0) < 1e-9


def test_dealt_shards_are_split_of_global_batch():
    """configs[3] shards: each rank's dealt_uniform_batch == split_batch of the one global batch"""
    glob = synth.dealt_uniform_batch(1000, 256, 7, seed=99, world=1, rank=0)
    for world in (2, 3, 4):
        for r in range(world):
            part = synth.dealt_uniform_batch(1000, 256, 7, seed=99, world=world, rank=r)
            w, off, mine = shard.split_batch(glob["wire"], glob["seg_off"], world, r)
            assert np.array_equal(mine, part["segments"])
            assert np.array_equal(off, part["seg_off"]) and np.array_equal(w, part["wire"])
    # the headers/masks decode like any other batch: the numpy restatement unmasks the payload
    ref = synth.unmask_reference(glob["wire"], glob["payload_off"], glob["plen"], glob["mask"])
    assert np.array_equal(synth.unmask_uniform(glob), ref)


def _bench(*args, env_extra=None):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=env, cwd=root)
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_gpus_n_launches_n_ranks():
    """`bench.py --gpus 2` (the driver's BENCH form, no launcher) must start 2
    ranks itself -- before touching a GPU -- and report n_gpus == 2; the dry run exercises the
    launch, the gloo process group, the barrier and the max-over-ranks time without device work"""
    rc, out, err = _bench("--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run")
    assert rc == 0, err[-2000:]
    assert out["n_gpus"] == 2 and out["rank_sum"] == 1, out     # ranks 0 and 1 both took part


def test_bench_world_size_mismatch_fails():
    """under a launcher whose world size differs from --gpus, the bench refuses to run"""
    rc, out, err = _bench("--gpus", "4", "--steps", "1", "--warmup", "0", "--dry-run",
                          env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc == 2 and out is None and "WORLD_SIZE=2" in err
