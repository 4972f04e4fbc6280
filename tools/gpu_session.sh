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
#   rlprof     the same under rocprofv3 --kernel-trace --stats -> gpurun_out/rlprof_TAG/
#   pmcrows    tools/pmc_rows.py (PMC bytes + VALU busy of the named low-roofline kernels)
#   py:FILE    python FILE (a tools/ script), e.g. py:tools/dropin_latency.py
#   ab:NAME    same-box A/B, alternating processes, ROUNDS (default 2) rounds of each side:
#              this library against federated_amd/lib_prev/libcfa.so (built from an earlier commit) for
#                rooflines  tools/kernel_rooflines.py
#                store      the bench line (no baselines), kernel_rooflines.py, slice_shape.py ring rounds
#                           at the N > 1 slice sizes
#                shape      slice_shape.py at K = 2/4/8/16 and K = 8 on scattered rows, and
#                           pipeline_threshold.py --native-only (the drop-in host pipeline)
#                pool       pipeline_threshold.py --native-only, 6 rounds, sides alternating who goes first
#              and, both sides on this library, a switch against its default:
#                signal     tools/dropin_latency.py vs --signal-off (completion word vs stream sync)
#                signal_c3  tools/probe/c3_calls.py vs --signal-off (config 3's CFA-GE calls)
#   bench:ARGS python bench.py ARGS, ARGS comma-separated (e.g. bench:--gpus,2,--params,1000000):
#              N > 1 self-launches its ranks (on a one-GPU box they share the card); the bench's own
#              statuses 3 (headline transport fallback) and 5 (an extra leg failed) printed a line
#              and do not end the session
# A fault, abort, time limit or any non-zero exit ends the session: no further GPU work.
set -u
TAG=${1:?tag}; shift
OUT=gpurun_out; mkdir -p "$OUT"; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
BENCH="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic --no-e2e --placement-leg 0"  # the headline alone
OKRC=" 0 "
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/${TAG}_$name.log" | cut -c1-400
  case "$OKRC" in *" $rc "*) ;; *) echo "!! stop"; exit $rc ;; esac
}
NB=0
ROUNDS=${ROUNDS:-2}
# one side of an A/B preset: ab_side PRESET SIDE ROUND (SIDE new|prev: the library; on|off: the switch)
ab_side() {
  local p=$1 side=$2 r=$3 lib=()
  [ "$side" = prev ] && lib=(env CFA_LIB="$PWD/federated_amd/lib_prev/libcfa.so")
  case "$p" in
    rooflines) step "ab_rl_${side}_$r" 300 "${lib[@]}" python tools/kernel_rooflines.py ;;
    store)
      step "ab_bench_${side}_$r" 200 "${lib[@]}" python $BENCH
      step "ab_rl_${side}_$r" 300 "${lib[@]}" python tools/kernel_rooflines.py
      step "ab_slice_${side}_$r" 200 "${lib[@]}" env SLICE_SIZES=1000000,3125056,6250048,12500000 SLICE_BPC=1 \
        SLICE_VEC=1 SLICE_CANDIDATES=2 SLICE_PASSES=5 SLICE_HALF=4 python tools/probe/slice_shape.py ;;
    shape)
      for h in 1 2 4 8; do
        step "ab_shape_k$((2 * h))_${side}_$r" 200 "${lib[@]}" env SLICE_SIZES=500000,1000000,2000000,3125056,6250048,9000000 \
          SLICE_BPC=1 SLICE_VEC=1 SLICE_CANDIDATES=2 SLICE_PASSES=5 SLICE_HALF=$h python tools/probe/slice_shape.py
      done
      step "ab_shape_k8s_${side}_$r" 200 "${lib[@]}" env SLICE_SIZES=500000,1000000,2000000,3125056,6250048,9000000 \
        SLICE_BPC=1 SLICE_VEC=1 SLICE_CANDIDATES=2 SLICE_PASSES=5 SLICE_HALF=4 SLICE_PATTERN=scattered \
        python tools/probe/slice_shape.py
      step "ab_pipe_${side}_$r" 200 "${lib[@]}" python tools/probe/pipeline_threshold.py --native-only ;;
    pool) step "ab_pipe_${side}_$r" 200 "${lib[@]}" python tools/probe/pipeline_threshold.py --native-only ;;
    signal) step "ab_signal_${side}_$r" 120 python tools/dropin_latency.py $([ "$side" = off ] && echo --signal-off) ;;
    signal_c3) step "ab_signal_c3_${side}_$r" 120 python tools/probe/c3_calls.py $([ "$side" = off ] && echo --signal-off) ;;
    *) echo "unknown A/B preset $p"; exit 2 ;;
  esac
}
ab() {
  local p=$1 n=$ROUNDS a=new b=prev
  [ "$p" = pool ] && n=6
  case "$p" in signal|signal_c3) a=on; b=off ;; esac
  for r in $(seq 1 "$n"); do
    if [ $((r % 2)) -eq 0 ] && [ "$p" = pool ]; then ab_side "$p" $b $r; ab_side "$p" $a $r
    else ab_side "$p" $a $r; ab_side "$p" $b $r; fi
  done
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
    rlprof) step rlprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/rlprof_$TAG" -o rl --output-format csv -- python3 tools/kernel_rooflines.py ;;
    pmcrows) step pmcrows 900 python tools/pmc_rows.py --out "$OUT/pmc_rows_$TAG" ;;
    py:*) f=${s#py:}; step "$(basename "$f" .py)" 600 python "$f" ;;
    ab:*) ab "${s#ab:}" ;;
    bench:*) NB=$((NB + 1)); a=${s#bench:}; a=${a//,/ }; OKRC=" 0 3 5 "
             step "bench$NB" 560 python bench.py $a; OKRC=" 0 "
             sed -i "1i # bench.py $a" "$OUT/${TAG}_bench$NB.log" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done"
