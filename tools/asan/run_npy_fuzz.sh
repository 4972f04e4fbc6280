#!/usr/bin/env bash
# Builds the numpy .npy / .npz reader with AddressSanitizer + UBSan (host code only, g++) and fuzzes
# it with mutations of files np.save / np.savez write (the TF2 exchange's model and status files).
# Usage: tools/asan/run_npy_fuzz.sh [iters per seed]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
# Scratch on tmpfs, one directory per run: the harness rewrites its file thousands of times, which
# blocks on a slow disk, and concurrent runs must not share it.
OUT=$(mktemp -d /dev/shm/cfa_npy_fuzz.XXXXXX)
trap 'rm -rf "$OUT"' EXIT
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer \
    -I"$ROOT/include" "$ROOT/federated_amd/csrc/cfa_npy.cpp" "$ROOT/tools/asan/npy_fuzz.cpp" \
    -o "$OUT/npy_fuzz"
python3 - "$OUT" <<'PY'
import pickle
import sys
import numpy as np
out = sys.argv[1]
rng = np.random.default_rng(0)
w = np.empty(4, dtype=object)
for i, s in enumerate([(3, 3, 1, 4), (4,), (20, 6), (6,)]):
    w[i] = rng.standard_normal(s).astype(np.float32)
w[2] = np.asfortranarray(w[2])
np.save(f"{out}/seed_model.npy", w, allow_pickle=True)
with open(f"{out}/seed_model_p3.npy", "wb") as f:  # numpy 1.x layout: protocol 3, GLOBAL opcodes
    np.lib.format.write_array_header_1_0(f, np.lib.format.header_data_from_array_1_0(w))
    pickle.dump(w, f, protocol=3)
np.savez(f"{out}/seed_status.npz", frame_count=70000, epoch_loss_history=[0.5, 0.25], training_end=False,
         epoch_count=3, loss=0.125)
np.save(f"{out}/seed_numeric.npy", np.arange(24, dtype=np.int16).reshape(2, 3, 4))
PY
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    "$OUT/npy_fuzz" "${1:-20000}" "$OUT"/seed*.np?
