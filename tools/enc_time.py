"""Encode timing (bench.py encode_configs: 64 KiB and 1 KiB echo batches), for kernel traces:
rocprofv3 --kernel-trace --stats -- python3 tools/enc_time.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from netman_amd import codec as K, synth  # noqa: E402

print(json.dumps(bench.encode_configs(torch, K, synth)))
