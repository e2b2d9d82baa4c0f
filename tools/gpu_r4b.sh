#!/bin/bash
# round-4: what async costs and buys at N=1 -- headline-config loss trajectories of local, plain
# AsySG-InCon (model / bucket granularity) and the look-ahead variants; same-box bench A/B of the
# publication granularity, the in-launch weight-gradient reduction, the bn2-only BN prologue and
# the Python GC setting (interleaved twice); the stall probe with and without gc.freeze()
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "topk_small or topk_exact or codec" > $O/ktests.log 2>&1 || { tail -30 $O/ktests.log; exit 1; }
tail -1 $O/ktests.log
timeout -k 10 600 python -u tools/trajectory.py --headline --runs local,async,async_la,async_bucket,async_bucket_la \
  --out $O/traj_headline.json > $O/traj.log 2>&1 || { tail -30 $O/traj.log; exit 1; }
run() {  # name, env...
  local name=$1; shift
  timeout -k 10 300 env "$@" python bench.py --steps 30 --warmup 5 --out $O/ab_$name.json > $O/ab_$name.log 2>&1 || { tail -20 $O/ab_$name.log; return 1; }
  python -c "import json;d=json.load(open('$O/ab_$name.json'));print('$name', d['value'], d['ms_per_step'], d['final_loss'], d['ps_staleness_mean'])"
}
for r in 1 2; do
  run base_r$r HIPPS_X=0 || exit 1
  run gcdefault_r$r HIPPS_X=0 BENCH_GC=default || exit 1
  run bucket16_r$r HIPPS_PS_GRANULARITY=bucket HIPPS_BUCKET_MB=16 || exit 1
  run wgred_off_r$r HIPPS_WGRAD_FUSED_REDUCE=0 || exit 1
  run bnpro2_r$r HIPPS_BN_PRO=2 || exit 1
done
STALL_OUT=$O/stall_gcdefault BENCH_ARGS="--gc default" bash tools/gpu_stall.sh > /dev/null || exit 1
STALL_OUT=$O/stall_gcfreeze BENCH_ARGS="--gc freeze" bash tools/gpu_stall.sh > /dev/null || exit 1
head -60 $O/stall_gcdefault/stalls.txt
