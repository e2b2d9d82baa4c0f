#!/bin/bash
# round-4: long-run allocator stability of the final build (200 steady steps) and the tuner's
# per-layer choices
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 400 python -u tools/alloc_probe.py --out $O/alloc_probe_200.txt --steps 200 --warmup 5 > $O/alloc_probe_200.log 2>&1 || { tail -20 $O/alloc_probe_200.log; exit 1; }
head -14 $O/alloc_probe_200.txt
timeout -k 10 300 python tools/tuner_dump.py --out $O/tuner.json > $O/tuner.log 2>&1 || { tail -20 $O/tuner.log; exit 1; }
python -c "import json;d=json.load(open('$O/tuner.json'));print(len(d['rows']), 'keys, sum', round(d['sum_ms'], 3), 'ms')"
