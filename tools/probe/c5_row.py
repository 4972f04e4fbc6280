"""Config 5 functional row only (tools/bench_configs.py population(): radar CNN buckets,
128 devices, v4 ring N=1, one CSR population launch per round)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))                    # tools/
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))   # repo root
import bench_configs as b  # noqa: E402

T = b.T
print(json.dumps({"config": "C5 radar CNN, 128 devices, ring (v4 N=1), one population launch",
                  **b.population(128, 24_622, T.ring_v4(128, 1), T.alphas_tf2)}), flush=True)
