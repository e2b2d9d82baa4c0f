#!/bin/bash
# weight gradients on a side stream: GPU test, then same-box A/B (default vs HIPPS_WGRAD_STREAM=1), interleaved
set -o pipefail
O=gpurun_out/ab_wgs
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread \
  tests/test_ps_async_gpu.py::test_gpu_wgrad_side_stream_bitwise > $O/test.log 2>&1 || { echo "test failed"; tail -30 $O/test.log; exit 1; }
grep -a "run-to-run\|passed\|failed" $O/test.log
run() {
  name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --out $O/$name.json > $O/$name.log 2>&1 || { echo "bench $name failed"; tail -20 $O/$name.log; return 1; }
  python3 -c "import json; r=json.load(open('$O/$name.json')); print('$name', r['value'], r['ms_per_step'])"
}
for rep in 1 2; do
  run base_$rep HIPPS_AB=1 &&
  run side_$rep HIPPS_WGRAD_STREAM=1 || exit 1
done
