"""The compact host path alone (bench.host_path_compact), for rocprofv3:
rocprofv3 --kernel-trace --memory-copy-trace --stats -- python3 tools/host_path_prof.py"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--groups", type=int, default=1_000_000)
ap.add_argument("--host-passes", type=int, default=4)
ap.add_argument("--host-partitions", type=int, default=2)
a = ap.parse_args()
print(json.dumps(bench.host_path_compact(a, 3, 0)))
a.host_partitions = 1
print(json.dumps(bench.host_path_compact(a, 3, 0)))
