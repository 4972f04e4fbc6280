"""Launch-shape sweep of the fp32 FedAvg divisor fold (cfa_mix_seq_div_f32, n = 8, P = 25M):
one process per (CFA_BLOCKS_PER_CU, CFA_VEC_PER_LANE) setting, since the library reads its
launch defaults once. Prints one JSON line per setting. GPU box: python tools/probe/div_sweep.py"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, sys, torch
sys.path.insert(0, ".")
from federated_amd.engine import get_engine
eng = get_engine(0)
P, n = 25_000_000, 8
g = torch.Generator(device="cuda").manual_seed(1)
local = torch.randn(P, device="cuda", generator=g)
nbrs = [torch.randn(P, device="cuda", generator=g) for _ in range(n)]
out = torch.empty(P, device="cuda")
for _ in range(5):
    eng.mix_seq_div(out, local, nbrs, [1.0] * n, [9.0] * n)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    eng.mix_seq_div(out, local, nbrs, [1.0] * n, [9.0] * n)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 50
print(json.dumps({"avg_launch_ms": round(ms, 4), "GBps": round((n + 2) * P * 4 / ms / 1e6, 1)}))
'''


def main():
    for bpc in (2, 3, 4, 6, 8):
        for vec in (1, 2, 4):
            env = dict(os.environ, CFA_BLOCKS_PER_CU=str(bpc), CFA_VEC_PER_LANE=str(vec))
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=120)
            line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else None
            row = {"kernel_entry": "cfa_mix_seq_div_f32", "n": 8, "blocks_per_cu": bpc, "vec_per_lane": vec}
            row.update(json.loads(line) if line else {"error": r.stderr[-300:]})
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
