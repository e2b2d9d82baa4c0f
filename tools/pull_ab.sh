set -o pipefail
mkdir -p gpurun_out/pullab
for f in 0 1; do for g in 1 4 16; do
HIPPS_PULL_FENCE=$f HIPPS_PULL_GRID_DIV=$g timeout -k 10 100 python -u bench/comm_bench.py --sizes-mb 16,51,102 --iters 20 > gpurun_out/pullab/f${f}_g${g}.log 2>&1 || exit 1
done; done
grep -h pull_kernel gpurun_out/pullab/*.log
