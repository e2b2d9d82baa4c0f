#!/bin/bash
# SQ counters of single gemm2 kernels (tools/g2_one.py), one rocprofv3 --pmc pass each, and a
# summary (wait / LDS-wait share of wave cycles, MFMA busy share of busy cycles)
#   bash tools/diag/g2_pmc.sh <out>
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-g2pmc5}
mkdir -p $O
CTR="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
run() {
  name=$1; shift
  timeout -k 10 120 python3 tools/g2_one.py "$@" > $O/$name.time 2>&1 || return 1
  echo "$name: $(cat $O/$name.time)"
  timeout -s KILL 90 rocprofv3 --pmc $CTR --output-format csv -d $O/$name -o pmc -- python3 tools/g2_one.py "$@" --iters 5 > $O/$name.log 2>&1 || return 1
}
run conv64 conv 64,56,64,1 --tile 128x64 &&
run conv128 conv 128,28,128,1 --tile 128x128 &&
run conv256 conv 256,14,256,1 --tile 256x256 &&
run conv256pp conv 256,14,256,1 --tile 256x256 --stages 5 &&
run wg0 wgrad 128,28,128,1,3 --cfg 0 &&
run wg2 wgrad 256,14,256,1,3 --cfg 2 &&
run gemm256 gemm 65536,4096,4096 --tile 256x256 --iters 10 &&
run gemm256pp gemm 65536,4096,4096 --tile 256x256 --stages 5 --iters 10 &&
python3 tools/diag/pmc_summary.py $O > $O/summary.txt && cat $O/summary.txt
