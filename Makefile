# Developer entry points (reference Makefile:1-198 equivalents).
IMG ?= ollama-operator-amd/operator:latest
SERVER_IMG ?= ollama-operator-amd/server:latest
PY ?= python3

.PHONY: build test test-gpu manifests bench bench-apply asan fuzz docker-build docker-push install uninstall deploy undeploy run
build:            ## compile the gfx950 HIP kernels + native runtime in-tree
	$(PY) build_native.py
test:             ## CPU test suite (the driver's `-m "not gpu"` run)
	$(PY) -m pytest tests -x -q -m "not gpu"
test-gpu:         ## GPU test suite (needs an MI355X)
	$(PY) -m pytest tests -x -q -m gpu
manifests:        ## regenerate deploy/ (CRD, RBAC, manager, samples, dist/install.yaml)
	$(PY) -m ollama_operator_amd.operator.manifests deploy
bench:            ## headline benchmark (1 GPU)
	$(PY) bench.py
bench-apply:      ## CRD apply -> Model Available, real processes (Phi-2 Q4_0 size, CPU or GPU)
	$(PY) scripts/bench_apply_ready.py --preset phi2 --ftype q4_0 --name phi
asan:             ## host AddressSanitizer + UBSan build of the native GGUF loader (csrc/tools)
	g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer \
	    csrc/tools/gguf_fuzz_main.cpp csrc/gguf/gguf.cpp -Icsrc -lpthread -o build/gguf_fuzz_asan
fuzz: asan        ## mutated-GGUF corpus through the Python reader and the ASan-built native loader
	$(PY) -m pytest tests/test_gguf_fuzz.py -q
docker-build:
	docker build -f docker/operator.Dockerfile -t $(IMG) .
	docker build -f docker/server.Dockerfile -t $(SERVER_IMG) .
docker-push:
	docker push $(IMG) && docker push $(SERVER_IMG)
install:          ## install the CRD into the current cluster
	kubectl apply -f deploy/config/crd/bases/ollama.ayaka.io_models.yaml
uninstall:
	kubectl delete -f deploy/config/crd/bases/ollama.ayaka.io_models.yaml
deploy:           ## install everything (namespace ollama-operator-system)
	kubectl apply -f deploy/dist/install.yaml
undeploy:
	kubectl delete -f deploy/dist/install.yaml
run:              ## run the operator against the current kubeconfig
	$(PY) -m ollama_operator_amd.operator --health-probe-bind-address=:8081 --metrics-bind-address=:8080
