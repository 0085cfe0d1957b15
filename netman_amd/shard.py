"""Multi-GPU sharding for the batched decoder.

Connections are independent: connection c's byte stream stays on one device (its header chain,
carry-over and reassembly are sequential per connection), so a batch shards by connection
segment with NO collective on the data path.  One process per GPU (torchrun); torch.distributed
is used only for the start barrier and the max-over-ranks step time.
"""
from __future__ import annotations

import os

import numpy as np


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_seed(base: int, rank: int) -> int:
    """per-rank generator seed for synthetic shards (disjoint streams per rank)"""
    return base + 1000 * rank


def assign_segments(n_segs: int, world: int) -> np.ndarray:
    """connection segment -> rank, round-robin (connection c -> GPU c mod world)"""
    return np.arange(n_segs, dtype=np.int64) % world


def split_batch(wire: np.ndarray, seg_off: np.ndarray, world: int, rank: int):
    """this rank's connections, re-packed as a contiguous batch (host side)"""
    owner = assign_segments(len(seg_off) - 1, world)
    mine = np.nonzero(owner == rank)[0]
    lens = (seg_off[mine + 1] - seg_off[mine]).astype(np.uint64)
    off = np.zeros(len(mine) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    parts = [wire[int(seg_off[i]):int(seg_off[i + 1])] for i in mine]
    out = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return out, off, mine


def max_over_ranks(x: float, dist=None, device=None) -> float:
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_rate(payload_bytes_per_rank, seconds_max: float, steps: int) -> float:
    """whole-job GiB/s: all ranks' payload / the slowest rank's time"""
    return float(np.sum(payload_bytes_per_rank)) * steps / seconds_max / 2**30
