#!/bin/bash
# GEMM core probe: shape table (tools/gemm_probe.py) + SQ counters on one compute-bound shape.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/gemm}
SHAPE=${SHAPE:-50176,1024,512}
mkdir -p $O
timeout -k 10 300 python tools/gemm_probe.py --out $O/probe.json > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_LDS \
  --output-format csv -d $O/sq -o sq -- python3 tools/gemm_probe.py --shape $SHAPE --iters 10 > $O/sq.log 2>&1
rc=$?
tail -n 3 $O/sq.log
exit $rc
