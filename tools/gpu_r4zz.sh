#!/bin/bash
# round-4 closing validation on a fresh box: the whole GPU suite, smoke(), the N=1 headline (with
# the fc layer on the shadow Linear, and an interleaved A/B without it), a steady-state kernel
# table, and the transformer configs
set -o pipefail
O=gpurun_out/r4zz
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -40 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
run() { name=$1; shift; timeout -k 10 300 python -u bench.py "$@" --out $O/$name.json > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }; python -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'], d.get('final_loss'))"; }
run bench_n1_r1 || exit 1
HIPPS_SHADOW_LINEAR=0 run bench_fc0_r1 || exit 1
run bench_n1_r2 || exit 1
HIPPS_SHADOW_LINEAR=0 run bench_fc0_r2 || exit 1
STEPS=12 bash tools/gpu_prof.sh > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
cp gpurun_out/prof/steady.txt $O/steady.txt
head -12 $O/steady.txt
run bert --model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec bf16 --steps 15 --warmup 5 || exit 1
run bert_thr --model bert-base --batch 32 --seq 512 --bucket-mb 4 --lr 1e-3 --codec threshold:1e-3:0.05 --steps 15 --warmup 5 || exit 1
run llama1b --model llama3-1b --batch 4 --seq 2048 --param-wire bf16 --lr 1e-3 --steps 10 --warmup 3 || exit 1
run llama8b --model llama3-8b --batch 1 --seq 2048 --param-wire bf16 --momentum 0 --lr 1e-4 --steps 6 --warmup 2 || exit 1
