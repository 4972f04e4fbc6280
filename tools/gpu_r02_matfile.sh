#!/usr/bin/env bash
# Round-2 GPU session: the drop-in golden replays and host-path GPU tests with the native MAT
# codec in the exchange, then the C1-C3 drop-in call latencies (native vs scipy file IO).
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
step configs_dropin 300 python tools/bench_configs.py dropin
step dropin 200 python tools/dropin_latency.py
echo "== done"
