#!/bin/bash
# One parameterised GPU recipe (replaces the round-4 one-off gpu_r4*.sh files).
#
#   bash tools/gpu.sh <out-dir under gpurun_out> <step> [<step> ...]
#
# steps (each under its own `timeout -k 10`, chained: the first failure ends the call):
#   tests            pytest -m gpu (thread timeout per test)       -> gpu_tests.log
#   tests:<expr>     pytest -m gpu -k <expr>
#   smoke            __graft_entry__.smoke()
#   bench            bench.py N=1, 30 timed steps                   -> bench_n1.json
#   bench2           bench.py N=1 twice more (box spread)           -> bench_n1_{b,c}.json
#   prof             rocprofv3 --kernel-trace --stats of bench.py, steady-state table -> steady.txt
#   reh_r50:<n>      driver launch rehearsal, n ranks sharing cuda:0 (gloo), ResNet-50 batch 64
#   reh_bert:<n>     ... BERT-base (seq 512, batch 4, 4 MB buckets)
#   reh_llama1b:<n>  ... Llama-3-1B (seq 1024, batch 1)
#   ipcprobe         tools/ipc_probe.py (concurrent IPC imports on one device)
#   configs          the secondary BASELINE configs at N=1 (top-k+int8, int8, fp32, BERT, Llama-1B)
#   llama8b          config 5 (Llama-3-8B seq 2048 batch 1) at N=1
#   emu7             bench.py --emulate-remote 7 and a plain N=1 row on the same box
#   codec            bench/codec_bench.py
#   tuner            tools/tuner_dump.py after a bench (which layers chose which kernel)
#   g2probe          tools/gemm2_probe.py (every gemm2 tile vs the first core / hipBLASLt / MIOpen)
#   scale8           ONLY on an 8-GPU node (never on the one-GPU pool): tests/test_multigpu.py with
#                    one rank per device (W = every device; the cross-device bitwise parity, chunked
#                    mailbox and W=8-geometry cases), then bench.py at N = 2, 4, 8 under
#                    torch.distributed.run -> scale_n{2,4,8}.json
#
# Extra bench.py arguments for bench/prof: BENCH_ARGS; env for every step is inherited.
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
fail() { echo "FAILED: $1"; tail -40 "$2"; exit 1; }

reh() {  # name n port args...
  local name=$1 n=$2 port=$3; shift 3
  HIPPS_BACKEND=gloo BENCH_HANG_DUMP=200 timeout -k 10 230 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port "$port" bench.py --gpus "$n" "$@" \
    --out "$OUT/$name.json" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -h "mailbox mapped" "$OUT/$name.log" | cut -c1-200
  [ $rc -eq 0 ] && cut -c1-300 "$OUT/$name.json" || fail "$name" "$OUT/$name.log"
}

for step in "$@"; do
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  case "$step" in
    tests|tests:*)
      K=()
      [ -n "$arg" ] && K=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${K[@]}" \
        > "$OUT/gpu_tests.log" 2>&1 || fail tests "$OUT/gpu_tests.log"
      tail -1 "$OUT/gpu_tests.log" ;;
    scale8)
      ndev=$(python -c "import torch; print(torch.cuda.device_count())")
      if [ "$ndev" -lt 8 ]; then echo "scale8: needs an 8-GPU node (found $ndev devices)"; exit 2; fi
      timeout -k 10 1800 python -u -m pytest tests/test_multigpu.py -v --timeout 600 --timeout-method thread \
        > "$OUT/multigpu_tests.log" 2>&1 || fail multigpu "$OUT/multigpu_tests.log"
      tail -1 "$OUT/multigpu_tests.log"
      for n in 2 4 8; do
        timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
          --master-port $((29700 + n)) bench.py --gpus "$n" --steps 20 --warmup 5 --out "$OUT/scale_n$n.json" \
          > "$OUT/scale_n$n.log" 2>&1 || fail "scale n=$n" "$OUT/scale_n$n.log"
        cut -c1-200 "$OUT/scale_n$n.json"
      done ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || fail smoke "$OUT/smoke.log"
      tail -1 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 300 python bench.py --steps 30 --warmup 8 $BENCH_ARGS --out "$OUT/bench_n1.json" \
        > "$OUT/bench.log" 2>&1 || fail bench "$OUT/bench.log"
      cut -c1-300 "$OUT/bench_n1.json" ;;
    bench2)
      for k in b c; do
        timeout -k 10 300 python bench.py --steps 30 --warmup 8 $BENCH_ARGS --out "$OUT/bench_n1_$k.json" \
          > "$OUT/bench_$k.log" 2>&1 || fail bench2 "$OUT/bench_$k.log"
        cut -c1-200 "$OUT/bench_n1_$k.json"
      done ;;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/hprof -o bench \
        -- python3 "$ROOT/bench.py" --steps 12 --warmup 5 $BENCH_ARGS) > "$OUT/bench_prof.log" 2>&1 \
        || fail prof "$OUT/bench_prof.log"
      T=$(find /tmp/hprof -name "bench_kernel_trace.csv" | head -1)
      python3 tools/steady_profile.py "$T" "$OUT/steady.txt" --skip 5 --title "ResNet-50 bs256 ps_async bf16 N=1 $BENCH_ARGS" ${PROF_DETAIL:+--detail "$PROF_DETAIL"}
      head -12 "$OUT/steady.txt" ;;
    reh_r50:*) reh "r50_n$arg" "$arg" $((29610 + arg)) --batch 64 --steps 10 --warmup 3 ;;
    reh_bert:*) reh "bert_n$arg" "$arg" $((29620 + arg)) --model bert-base --batch 4 --seq 512 --bucket-mb 4 \
                  --lr 1e-3 --steps 8 --warmup 3 ;;
    reh_llama1b:*) reh "llama1b_n$arg" "$arg" $((29630 + arg)) --model llama3-1b --batch 1 --seq 1024 \
                     --lr 1e-3 --steps 6 --warmup 2 ;;
    ipcprobe|ipcprobe:*)  # ipcprobe[:chunk_mb] -- 2 importers, regions 256 MB .. 8 GB, twice
      HIPPS_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 \
        --master-addr 127.0.0.1 --master-port 29655 tools/ipc_probe.py --sizes 256,1024,2048,4096,8192 \
        --repeat 2 --chunk-mb "${arg:-0}" > "$OUT/ipc_probe_c${arg:-0}.txt" 2>&1 \
        || fail ipcprobe "$OUT/ipc_probe_c${arg:-0}.txt"
      grep -v "amdgpu.ids\|socket.cpp" "$OUT/ipc_probe_c${arg:-0}.txt" | tail -12 ;;
    ipclog)  # one importer with AMD_LOG_LEVEL=4 on 4 and 8 GB regions (runtime log of a slow import)
      AMD_LOG_LEVEL=4 HIPPS_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29656 tools/ipc_probe.py --sizes 4096,8192 \
        --limit 30 > "$OUT/ipc_log.txt" 2>&1 || { grep -v "amdgpu.ids" "$OUT/ipc_log.txt" | grep -i "ipc\|TIMEOUT\|rank\|region" | tail -40; fail ipclog "$OUT/ipc_log.txt"; }
      grep -i "region" "$OUT/ipc_log.txt" | tail -5 ;;
    configs)
      for c in "topk_int8:0.01" int8 fp32; do
        n=$(echo "$c" | tr ':.' '__')
        timeout -k 10 300 python bench.py --steps 20 --warmup 6 --codec "$c" --out "$OUT/r50_$n.json" \
          > "$OUT/r50_$n.log" 2>&1 || fail "config $c" "$OUT/r50_$n.log"
        cut -c1-200 "$OUT/r50_$n.json"
      done
      timeout -k 10 300 python bench.py --model bert-base --batch 32 --seq 512 --lr 1e-3 --steps 10 --warmup 4 \
        --out "$OUT/bert.json" > "$OUT/bert.log" 2>&1 || fail bert "$OUT/bert.log"
      cut -c1-200 "$OUT/bert.json"
      timeout -k 10 300 python bench.py --model bert-base --batch 32 --seq 512 --lr 1e-3 --steps 10 --warmup 4 \
        --codec threshold:0.001 --bucket-mb 4 --out "$OUT/bert_thr.json" > "$OUT/bert_thr.log" 2>&1 \
        || fail bert_thr "$OUT/bert_thr.log"
      cut -c1-200 "$OUT/bert_thr.json"
      timeout -k 10 300 python bench.py --model llama3-1b --batch 4 --seq 2048 --param-wire bf16 --lr 1e-3 --steps 8 \
        --warmup 3 \
        --out "$OUT/llama1b.json" > "$OUT/llama1b.log" 2>&1 || fail llama1b "$OUT/llama1b.log"
      cut -c1-200 "$OUT/llama1b.json" ;;
    llama8b)
      timeout -k 10 600 python bench.py --model llama3-8b --batch 1 --seq 2048 --param-wire bf16 --momentum 0 \
        --lr 1e-4 --steps 6 --warmup 3 \
        --out "$OUT/llama8b.json" > "$OUT/llama8b.log" 2>&1 || fail llama8b "$OUT/llama8b.log"
      cut -c1-300 "$OUT/llama8b.json" ;;
    emu7)
      timeout -k 10 300 python bench.py --steps 30 --warmup 8 --out "$OUT/emu_base.json" > "$OUT/emu_base.log" 2>&1 \
        || fail emu_base "$OUT/emu_base.log"
      timeout -k 10 300 python bench.py --steps 30 --warmup 8 --emulate-remote 7 --out "$OUT/emu_er7.json" \
        > "$OUT/emu_er7.log" 2>&1 || fail emu7 "$OUT/emu_er7.log"
      cut -c1-160 "$OUT/emu_base.json" "$OUT/emu_er7.json" ;;
    codec)
      timeout -k 10 300 python bench/codec_bench.py --out "$OUT/codec_bench.json" > "$OUT/codec.log" 2>&1 \
        || fail codec "$OUT/codec.log"
      tail -30 "$OUT/codec.log" ;;
    tuner)
      timeout -k 10 300 python tools/tuner_dump.py --out "$OUT/tuner.json" > "$OUT/tuner.txt" 2>&1 \
        || fail tuner "$OUT/tuner.txt"
      tail -20 "$OUT/tuner.txt" ;;
    g2probe)
      timeout -k 10 400 python tools/gemm2_probe.py --out "$OUT/gemm2_probe.json" > "$OUT/g2probe.log" 2>&1 \
        || fail g2probe "$OUT/g2probe.log"
      python3 - "$OUT/gemm2_probe.json" <<'PY'
import json, sys
for r in json.load(open(sys.argv[1])):
    tf = {k[3:-3]: v for k, v in r.items() if k.startswith("g2_") and k.endswith("_TF") and k != "g2_best_TF"}
    ref = r.get("hipblaslt_TF") or r.get("miopen_TF")
    best = max(tf, key=tf.get)
    print({k: r[k] for k in ("M", "K", "N", "Cin", "H", "Cout", "stride") if k in r}, "best", best, tf[best],
          "ref", ref, "pp", tf.get("256x256s5"), "m32", tf.get("256x256s6"), "s2", tf.get("256x256s2"))
PY
      ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
