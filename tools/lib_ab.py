"""A/B of two builds of libwscodec.so on one box: loads the given library file instead of the
in-tree one, then runs a bench leg and prints its JSON.
    python tools/lib_ab.py <lib.so> encode|configs [name fragment ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from netman_amd import codec as K, synth  # noqa: E402

if __name__ == "__main__":
    K.load_library(os.path.abspath(sys.argv[1]))
    if sys.argv[2] == "encode":
        print(json.dumps(bench.encode_configs(torch, K, synth)))
    else:
        print(json.dumps(bench.other_configs(torch, K, synth, only=sys.argv[3:] or None)))
