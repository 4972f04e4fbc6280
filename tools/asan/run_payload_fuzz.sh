#!/usr/bin/env bash
# Builds the payload codec with AddressSanitizer + UBSan (host code only, g++) and fuzzes it with
# mutations of reference-shaped payloads written by CPython's pickle. Usage: tools/asan/run_payload_fuzz.sh [iters]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
# Scratch on tmpfs, one directory per run: the harness rewrites its file thousands of times, which
# blocks on a slow disk, and concurrent runs must not share it.
OUT=$(mktemp -d /dev/shm/cfa_payload_fuzz.XXXXXX)
trap 'rm -rf "$OUT"' EXIT
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -pthread \
    -I"$ROOT/include" "$ROOT/federated_amd/csrc/cfa_payload.cpp" "$ROOT/tools/asan/payload_fuzz.cpp" \
    -o "$OUT/payload_fuzz"
python3 - "$OUT" <<'PY'
import pickle, sys
import numpy as np
out = sys.argv[1]
rng = np.random.default_rng(0)
w = [rng.standard_normal(s).astype(np.float32) for s in [(3, 3, 1, 4), (4,), (20, 6), (6,)]]
d = {f"model_layer{k}": a.tolist() for k, a in enumerate(w)}
d.update(device=3, framecount=70000, local_epoch=-5, training_end=False)
for p in (2, 4, 5):
    open(f"{out}/seed{p}.pkl", "wb").write(pickle.dumps(d, protocol=p))
open(f"{out}/seed_nested.pkl", "wb").write(pickle.dumps({"a": [[[]], [[]]], "b": [[1, 2.5], [True, 0]], "s": [[0.5]] * 3}))
PY
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    "$OUT/payload_fuzz" "${1:-20000}" "$OUT"/seed*.pkl
