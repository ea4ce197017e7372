"""The C4 fp32 bench configuration alone (10M x 1024 fp32 samples,
k = 4096), for a per-iteration kernel trace of that line:
  rocprofv3 --kernel-trace --stats -d DIR -o run -- python tools/c4_f32_run.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main():
    import torch
    dev = torch.device("cuda", 0)
    r = bench.run_config(torch, None, dev, 0, 1, 10_000_000, 1024, 4096,
                         1_000_000, 4, 2, "auto", False, f32=True)
    print(json.dumps({k: v for k, v in r.items()
                      if isinstance(v, (int, float, str))}))


if __name__ == "__main__":
    main()
