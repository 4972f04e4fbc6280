#!/usr/bin/env bash
# One GPU-box session, parametrised by the steps to run (replaces round 2's per-session scripts).
#
#   bash tools/gpu_session.sh TAG STEP [STEP ...]
#
# Steps (each under its own time limit, output in gpurun_out/TAG_STEP.log):
#   tests      python -m pytest tests -m gpu -x (the driver's round-end command, with per-test timeouts)
#   tests:EXPR the same restricted by -k EXPR
#   smoke      __graft_entry__.smoke()
#   bench      the default bench line (CPU baselines, live PMC traffic)
#   rocprof    rocprofv3 --kernel-trace --stats of the bench command -> gpurun_out/prof_TAG/
#   fetch      rocprofv3 --pmc FETCH_SIZE of the bench command     -> gpurun_out/pmc_TAG/
#   write      rocprofv3 --pmc WRITE_SIZE of the bench command     -> gpurun_out/pmc_TAG/
#   rooflines  tools/kernel_rooflines.py (event-timed roofline of every streaming kernel)
#   pmcrows    tools/pmc_rows.py (PMC bytes + VALU busy of the named low-roofline kernels)
#   py:FILE    python FILE (a tools/ script), e.g. py:tools/dropin_latency.py
# A fault, abort, time limit or any non-zero exit ends the session: no further GPU work.
set -u
TAG=${1:?tag}; shift
OUT=gpurun_out; mkdir -p "$OUT"; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
BENCH="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic --no-e2e"
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/${TAG}_$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "!! stop"; exit $rc; fi
}
for s in "$@"; do
  case "$s" in
    tests) step pytest_gpu 1100 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu -p no:cacheprovider ;;
    tests:*) step pytest_sel 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu -p no:cacheprovider -k "${s#tests:}" ;;
    smoke) step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 500 python bench.py --steps 20 --warmup 5 ;;
    rocprof) step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 $BENCH ;;
    fetch) step fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_$TAG" -o fetch --output-format csv -- python3 $BENCH ;;
    write) step write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_$TAG" -o write --output-format csv -- python3 $BENCH ;;
    rooflines) step rooflines 500 python tools/kernel_rooflines.py ;;
    pmcrows) step pmcrows 900 python tools/pmc_rows.py --out "$OUT/pmc_rows_$TAG" ;;
    py:*) f=${s#py:}; step "$(basename "$f" .py)" 600 python "$f" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done"
