#!/usr/bin/env bash
# Round-2 GPU session: the drop-in golden replays (TF1 + TF2 + PS) with the native .mat and
# .npy/.npz readers in the exchange, then the TF2 / PS per-call costs (native reader vs np.load).
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "!! stop"; exit $rc; fi
}
step pytest_dropin 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_consensus_golden.py tests/test_gpu_variants_golden.py tests/test_tf1_models.py tests/test_gpu_population.py
step tf2_calls 300 python tools/probe/tf2_calls.py
echo "== done"
