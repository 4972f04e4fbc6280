#!/usr/bin/env bash
# Round-2 closing evidence: whole GPU suite, smoke, the default bench line (live PMC traffic),
# a rocprofv3 kernel-trace summary of the bench, the BASELINE configs, drop-in latency.
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "!! stop"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_n1 500 python bench.py --steps 20 --warmup 3
step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_final" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-live-traffic
step configs 600 python tools/bench_configs.py
step dropin 200 python tools/dropin_latency.py
echo "== done"
