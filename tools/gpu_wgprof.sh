#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/wgprof
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv1x1_gpu.py -x -q -k wgrad --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { echo "conv tests failed"; tail -60 gpurun_out/conv_tests.log; exit 1; }
tail -1 gpurun_out/conv_tests.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/wgp -o wg -- python3 $ROOT/tools/bench_conv1x1.py > $ROOT/gpurun_out/wgprof/bench.log 2>&1 || { echo "prof failed"; tail -20 $ROOT/gpurun_out/wgprof/bench.log; exit 1; }
cd $ROOT
cp $(find /tmp/wgp -name "wg_kernel_stats.csv" | head -1) gpurun_out/wgprof/
python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/wgprof/wg_kernel_stats.csv')))
for r in rows:
    n=r['Name']
    if 'wgrad' in n or 'conv1x1' in n or 'wrw' in n or 'SubTensor' in n or 'fill' in n.lower():
        print(r['Calls'], r['AverageNs'], n[:110])
"
