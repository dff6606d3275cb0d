# Developer entry points (reference: Makefile of the reference repo -- build, test,
# release-style targets).  GPU targets need an MI355X; everything else runs on a CPU box.
PY ?= python
JOBS ?= 6

.PHONY: build test test-gpu sanitize ci bench bench64 smoke clean docker wheel

build:            ## compile libmoosex.so (g++ host + hipcc gfx950) and the _moosert runtime
	$(PY) -c "import __graft_entry__ as g; g.build()"

test: build       ## CPU suite (gloo for the multi-process tests)
	$(PY) -m pytest tests -q -m "not gpu" -n $(JOBS)

test-gpu: build   ## GPU suite on an MI355X
	$(PY) -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread

sanitize:         ## host C++ under ASAN+UBSAN and TSAN
	scripts/sanitize.sh all

ci:               ## what CI runs: build, CPU suite, sanitizers
	scripts/ci.sh

smoke: build      ## one tiny replicated dot + sigmoid on cuda:0
	$(PY) __graft_entry__.py smoke

bench: build      ## headline benchmark (1 GPU; GPUS=N for N ranks)
	$(PY) bench.py --gpus $${GPUS:-1}

bench64: build
	$(PY) bench.py --gpus $${GPUS:-1} --ring 64

wheel: build
	$(PY) -m pip wheel --no-deps --no-build-isolation -w dist .

docker:
	docker build -t moose-amd .

clean:
	rm -rf build moose_amd/_native/*.so dist *.egg-info
