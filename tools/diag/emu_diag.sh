# A/B of the one-GPU rehearsal of remote workers' PS load (bench.py --emulate-remote): which part
# of it costs worker 0 -- the accumulator path (direct update off), the batched decode, or the
# emulated HBM traffic -- for the native and the Python PS loop.
set -o pipefail
O=gpurun_out/${1:-r5q}; mkdir -p $O
export HIPPS_HOST_TIMING=1 HIPPS_WAIT_DIAG=1
run() {  # name "ENV=v ..." bench-args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 6 "$@" --out $O/$name.json > $O/$name.log 2>&1 \
    || return 1
  echo "== $name $(grep -h 'host ms' $O/$name.log | cut -c1-150)"
  python3 -c "import json;d=json.load(open('$O/$name.json'));print(d['value'], d['ms_per_step'])"
}
case "${2:-all}" in
  stream)
    run er7_notraffic_nostream "HIPPS_EMU_TRAFFIC=0 HIPPS_EMU_STREAM=0" --emulate-remote 7 &&
    run er7_nostream "HIPPS_EMU_STREAM=0" --emulate-remote 7 &&
    run er7_nostream_py "HIPPS_EMU_STREAM=0 HIPPS_NATIVE_PS=0" --emulate-remote 7 &&
    run base "HIPPS_X=0" ;;
  accpool)  # the accumulator path (rank 0 at N > 1 for remote messages) with the pool advanced
    run nodirect_skip1 "HIPPS_PS_DIRECT=0 HIPPS_POOL_SKIP=1" && run nodirect_skip2 "HIPPS_PS_DIRECT=0 HIPPS_POOL_SKIP=2" &&
    run er7_default "HIPPS_X=0" --emulate-remote 7 && run base "HIPPS_X=0" ;;
  pool)  # the same model with the torch stream pool advanced k streams before the side stream
    run skip1 "HIPPS_POOL_SKIP=1" && run skip2 "HIPPS_POOL_SKIP=2" && run skip3 "HIPPS_POOL_SKIP=3" &&
    run skip4 "HIPPS_POOL_SKIP=4" && run base "HIPPS_X=0" ;;
  side)  # where the weight-gradient side stream lands once the extra stream exists
    run er7nt_stream "HIPPS_EMU_TRAFFIC=0 HIPPS_EMU_STREAM=1" --emulate-remote 7 &&
    run er7nt_stream_wgprio "HIPPS_EMU_TRAFFIC=0 HIPPS_EMU_STREAM=1 HIPPS_WGRAD_PRIO=-1" --emulate-remote 7 &&
    run er7nt_stream_nowgs "HIPPS_EMU_TRAFFIC=0 HIPPS_EMU_STREAM=1 HIPPS_WGRAD_STREAM=0" --emulate-remote 7 &&
    run base_wgprio "HIPPS_WGRAD_PRIO=-1" &&
    run base_nowgs "HIPPS_WGRAD_STREAM=0" &&
    run base "HIPPS_X=0" ;;
  queues)  # the extra emulation stream with 8 hardware queues per process instead of HIP's 4
    run er7_q8 "GPU_MAX_HW_QUEUES=8 HIPPS_EMU_STREAM=1" --emulate-remote 7 &&
    run base_q8 "GPU_MAX_HW_QUEUES=8" &&
    run er7_q4 "HIPPS_EMU_STREAM=1" --emulate-remote 7 &&
    run base "HIPPS_X=0" ;;
  *)
    run base "HIPPS_X=0" &&
    run nodirect "HIPPS_PS_DIRECT=0" &&
    run nodirect_py "HIPPS_PS_DIRECT=0 HIPPS_NATIVE_PS=0" &&
    run er7_notraffic "HIPPS_EMU_TRAFFIC=0" --emulate-remote 7 &&
    run er7 "HIPPS_X=0" --emulate-remote 7 ;;
esac
