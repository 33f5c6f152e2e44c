"""Print bench.py's drop-in latency rows (LJ v1, T' = 64 / 512 / 2048, B = 1 and 16) as JSON.
Usage (GPU box): python tools/latency.py [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    print(json.dumps(bench.latency_rows(torch.device("cuda:0"), reps)))
