set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_population.py -k "hostmixer or native" > $OUT/native_tests.log 2>&1 || { tail -30 $OUT/native_tests.log; exit 1; }
tail -2 $OUT/native_tests.log
timeout -k 10 400 python tools/probe/pipeline_threshold.py > $OUT/native_probe.log 2>&1; rc=$?; tail -c 3000 $OUT/native_probe.log; exit $rc
