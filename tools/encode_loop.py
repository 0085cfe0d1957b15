"""Device time of wsc_encode for the bench's two encode batches (median of 10, torch events):
    python tools/encode_loop.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from netman_amd import codec as K  # noqa: E402
from netman_amd import synth  # noqa: E402

if __name__ == "__main__":
    for k, v in bench.encode_configs(torch, K, synth).items():
        print(k, v["ms"], v["gb_s"], v["check_ok"])
