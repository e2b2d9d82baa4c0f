set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_stem_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stem_tests.log 2>&1; rc=$?; tail -2 gpurun_out/stem_tests.log; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/ab
for v in 1 0; do
  HIPPS_FUSED_STEMBWD=$v timeout -k 10 300 python bench.py --steps 30 --warmup 8 --out gpurun_out/ab/stembwd_$v.json > gpurun_out/ab/stembwd_$v.log 2>&1 || exit 1
  cut -c1-160 gpurun_out/ab/stembwd_$v.json
done
export TMPDIR=/tmp; ROOT=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/hp1 -o b -- python3 $ROOT/bench.py --steps 12 --warmup 5 > $ROOT/gpurun_out/ab/prof.log 2>&1 || exit 1
cd $ROOT && python3 tools/steady_profile.py $(find /tmp/hp1 -name "b_kernel_trace.csv" | head -1) gpurun_out/ab/steady_stembwd1.txt --skip 5 --title "stem fused bwd" && head -9 gpurun_out/ab/steady_stembwd1.txt && grep -E "stem|maxpool" gpurun_out/ab/steady_stembwd1.txt | cut -c1-120
