#!/usr/bin/env bash
# Builds the MATLAB level-5 codec with AddressSanitizer + UBSan (host code only, g++) and fuzzes
# its reader with mutations of files scipy.io.savemat writes (the TF1 exchange's model and gradient
# files). Usage: tools/asan/run_matfile_fuzz.sh [iters per seed]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
# Scratch on tmpfs, one directory per run: the harness rewrites its file thousands of times, which
# blocks on a slow disk, and concurrent runs must not share it.
OUT=$(mktemp -d /dev/shm/cfa_matfile_fuzz.XXXXXX)
trap 'rm -rf "$OUT"' EXIT
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer \
    -I"$ROOT/include" "$ROOT/federated_amd/csrc/cfa_matfile.cpp" "$ROOT/tools/asan/matfile_fuzz.cpp" \
    -o "$OUT/matfile_fuzz"
python3 - "$OUT" <<'PY'
import sys
import numpy as np
import scipy.io as sio
out = sys.argv[1]
rng = np.random.default_rng(0)
sio.savemat(f"{out}/seed_model.mat", {"weights1": rng.standard_normal((40, 8)).astype(np.float32),
            "biases1": np.ones(8, np.float32), "epoch": 3, "loss_sample": np.zeros(3), "counter_param": 1})
sio.savemat(f"{out}/seed_grad.mat", {"grad_weights1": rng.standard_normal((3, 3, 1, 4)),
            "grad_biases1": np.arange(4, dtype=np.int16), "u": np.uint8(7)})
PY
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    "$OUT/matfile_fuzz" "$OUT/fuzz.mat" "${1:-20000}" "$OUT"/seed*.mat
