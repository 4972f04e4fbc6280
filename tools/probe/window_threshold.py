"""Window passes vs the one-launch CSR kernel for a 32-device K = 4 window population across
bucket sizes: where topology.WINDOW_MIN_P should sit. GPU box:
python tools/probe/window_threshold.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import tools.bench_configs as bc  # noqa: E402
from federated_amd import topology as T  # noqa: E402


def main():
    lists = [[(d + o) % 32 for o in (-2, -1, 1, 2)] for d in range(32)]
    for P in (262_144, 1_071_748, 2_097_152, 4_000_000):
        for w in (False, True):
            r = bc.population(32, P, lists, T.alphas_tf2, use_window=w)
            print(json.dumps({"devices": 32, "K": 4, "P": P, "window": w,
                              **{k: r[k] for k in ("path", "round_us", "GBps", "round_us_graph")}}), flush=True)


if __name__ == "__main__":
    main()
