#!/bin/bash
# stem kernels: per-kernel times and SQ counters (one --pmc pass)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/stem_prof
mkdir -p $O
ROOT=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sp -o sp -- python3 $ROOT/tools/stem_probe.py > $ROOT/$O/trace.log 2>&1 || { tail -20 $ROOT/$O/trace.log; exit 1; }
cd $ROOT
cp $(find /tmp/sp -name "sp_kernel_stats.csv" | head -1) $O/kernel_stats.csv && cut -d, -f1-8 $O/kernel_stats.csv | head -8
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_LDS \
  -d $O/sq -o sq -- python3 tools/stem_probe.py --iters 4 > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
python3 tools/rocpd_pmc.py $(find $O/sq -name "*.db") --filter stem > $O/sq.txt && cat $O/sq.txt
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRDREQ_sum TCC_EA0_WRDREQ_64B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum \
  -d $O/tcc -o tcc -- python3 tools/stem_probe.py --iters 4 > $O/tcc.log 2>&1 || { tail -5 $O/tcc.log; exit 1; }
python3 tools/rocpd_pmc.py $(find $O/tcc -name "*.db") --filter stem > $O/tcc.txt && cat $O/tcc.txt
