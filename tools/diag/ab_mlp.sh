set -o pipefail
O=gpurun_out/ab_mlp; mkdir -p $O
for r in 1 2; do
for v in off on; do
  if [ $v = off ]; then E="HIPPS_GELU_MLP=0 HIPPS_RES_LINK=0"; else E=""; fi
  env $E timeout -k 10 300 python bench.py --model bert-base --batch 32 --seq 512 --lr 1e-3 --steps 20 --warmup 5 --out $O/bert_${v}_$r.json > $O/bert_${v}_$r.log 2>&1 || { echo fail $v; tail -20 $O/bert_${v}_$r.log; exit 1; }
  echo $v $r $(cut -c1-120 $O/bert_${v}_$r.json)
done; done
