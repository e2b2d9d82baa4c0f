# hipps developer targets (reference: Makefile `test: mpirun -n 2 py.test -s`).
# Multi-process tests spawn their own gloo worlds, so plain pytest replaces `mpirun -n 2`.
PY ?= python

.PHONY: build test test-gpu test-dist bench bench-codec clean

build:
	$(PY) -m hipps._build

test:
	$(PY) -m pytest tests -m "not gpu" -q

test-gpu: build
	$(PY) -m pytest tests -m gpu -q

# the reference's two-rank run, as a real launcher-started world (gloo on CPU)
test-dist:
	$(PY) -m hipps.launch -n 2 examples/train_mlp_ps.py --mode ps_sync --steps 20
	$(PY) -m hipps.launch -n 2 examples/train_mlp_ps.py --mode allgather --steps 20
	$(PY) -m hipps.launch -n 3 examples/train_mlp_ps.py --mode ps_async --steps 20

bench: build
	$(PY) bench.py

bench-codec: build
	$(PY) bench/codec_bench.py --out profiles/codec_bench.json

clean:
	$(PY) -m hipps._build --clean
