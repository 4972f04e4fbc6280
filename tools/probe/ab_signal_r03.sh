#!/usr/bin/env bash
# A/B of the drop-in completion: the signal word (default) against hipStreamSynchronize,
# alternating processes on one box (tools/dropin_latency.py). Output: gpurun_out/ab_signal.jsonl
set -u
OUT=gpurun_out; mkdir -p "$OUT"; cd "${GRAFT_REPO_ROOT:-.}"
for i in 1 2 3; do
  timeout -k 10 120 python tools/dropin_latency.py >> "$OUT/ab_signal.jsonl" || exit $?
  timeout -k 10 120 python tools/dropin_latency.py --signal-off >> "$OUT/ab_signal.jsonl" || exit $?
done
