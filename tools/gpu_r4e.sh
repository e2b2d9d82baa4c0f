#!/bin/bash
# round-4, default build: host cProfile of the timed steps, the stall probe, the steady kernel
# table, and same-box A/B of the publication granularity and the mailbox depth (interleaved twice)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 300 python -u tools/host_profile.py --out $O/host_profile.txt --steps 20 --warmup 5 > $O/host_profile.log 2>&1 || { tail -20 $O/host_profile.log; exit 1; }
head -45 $O/host_profile.txt
STALL_OUT=$O/stall bash tools/gpu_stall.sh > /dev/null || exit 1
head -40 $O/stall/stalls.txt
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/hprof_$$ -o bench -- python3 $ROOT/bench.py --steps 12 --warmup 5 > $ROOT/$O/bench_prof.log 2>&1 || { echo "prof failed"; tail -20 $ROOT/$O/bench_prof.log; exit 1; }
cd $ROOT
T=$(find /tmp/hprof_$$ -name "bench_kernel_trace.csv" | head -1)
python3 tools/steady_profile.py "$T" $O/steady.txt --skip 5 --title "ResNet-50 bs256 ps_async bf16 N=1 (round-4 defaults)" || exit 1
head -12 $O/steady.txt
ab() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 "$@" --out $O/ab_$name.json > $O/ab_$name.log 2>&1 || { tail -20 $O/ab_$name.log; return 1; }
  python -c "import json;d=json.load(open('$O/ab_$name.json'));print('$name', d['value'], d['ms_per_step'], d['final_loss'], d['ps_staleness_mean'])"
}
for r in 1 2; do
  ab default_r$r || exit 1
  ab model64_r$r --granularity model --bucket-mb 64 || exit 1
  ab slots32_r$r --mailbox-slots 32 || exit 1
  ab local_r$r --mode local || exit 1
done
for r in 1 2; do
  for pv in 2 1; do
    timeout -k 10 300 env HIPPS_BN_PRO=$pv python bench.py --steps 30 --warmup 5 --out $O/ab_bnpro${pv}_r$r.json > $O/ab_bnpro${pv}_r$r.log 2>&1 || { tail -20 $O/ab_bnpro${pv}_r$r.log; exit 1; }
    python -c "import json;d=json.load(open('$O/ab_bnpro${pv}_r$r.json'));print('bnpro$pv r$r', d['value'], d['ms_per_step'], d['final_loss'], d['ps_staleness_mean'])"
  done
done
