"""bench.py's encode lines alone (one JSON line)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from netman_amd import codec as K  # noqa: E402
from netman_amd import synth  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(bench.encode_configs(torch, K, synth)))
