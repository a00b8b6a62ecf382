# Native build + test entry points (the in-tree .so files are what the runtime loads).
PY ?= python

.PHONY: build build-asan test test-gpu manifests bench profile clean

build:            ## compile csrc/kernels/*.hip for gfx950 + the host C++ modules, in-tree
	$(PY) -m operator_amd._build -v

build-asan:       ## host C++ (pattern compiler / packer / scorer) with ASan + UBSan, fuzzed in a child process
	$(PY) -m pytest tests/test_sanitizers.py -q

test:             ## CPU tier (no GPU): controllers, patterns, reference ops, TP/DP over gloo, engine pool
	$(PY) -m pytest tests/ -x -q -m "not gpu"

test-gpu:         ## MI355X tier: kernel numerics vs fp32 references, scan, model, graphs
	$(PY) -m pytest tests/ -x -q -m gpu

manifests:        ## CRDs + RBAC + Deployment
	$(PY) -m operator_amd manifests --out operator_amd/api/manifests/podmortem-operator.yaml

bench:            ## flagship benchmark (one JSON line)
	$(PY) bench.py

profile:          ## kernel trace of a short flagship run (cd /tmp first: rocprofv3 scratch files)
	cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $(CURDIR)/gpurun_out/prof -o prof -- $(PY) $(CURDIR)/bench.py --steps 1 --warmup 1

clean:
	rm -rf build operator_amd/*.so
