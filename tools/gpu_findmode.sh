#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/fm
for fm in 1 3 5; do
  MIOPEN_FIND_MODE=$fm timeout -k 10 400 python bench.py --steps 20 --warmup 6 --out gpurun_out/fm/fm$fm.json > gpurun_out/fm/fm$fm.log 2>&1 || { echo "fm $fm failed"; tail -5 gpurun_out/fm/fm$fm.log; exit 1; }
  echo "find_mode=$fm $(python -c "import json;d=json.load(open('gpurun_out/fm/fm$fm.json'));print(d['value'], d['ms_per_step'])")"
done
