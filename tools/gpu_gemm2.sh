set -o pipefail
mkdir -p gpurun_out/g2
timeout -k 10 300 python -u tools/gemm2_probe.py --out gpurun_out/g2/probe.json > gpurun_out/g2/probe.log 2>&1; rc=$?
tail -25 gpurun_out/g2/probe.log
exit $rc
