# cron-operator (MI355X-first rebuild).  Target names follow the reference
# Makefile (Makefile:1-331) where the concept carries over; Go/controller-gen/
# envtest/kind steps become their Python/fake-apiserver equivalents.

VERSION ?= $(shell cat VERSION)
IMG_REGISTRY ?= docker.io
IMG_REPOSITORY ?= cron-operator-amd/cron-operator
IMG_TAG ?= $(patsubst v%,%,$(VERSION))
IMG ?= $(IMG_REGISTRY)/$(IMG_REPOSITORY):$(IMG_TAG)
# the MI355X payload image the examples/mi355x Crons run (Dockerfile.payload)
PAYLOAD_IMG ?= $(IMG_REGISTRY)/cron-operator-amd/cron-operator-mi355x-payload:$(IMG_TAG)
# the ROCm PyTorch base of the payload image: pin it to the release your nodes' driver supports
ROCM_PYTORCH_IMAGE ?= rocm/pytorch:latest
CONTAINER_TOOL ?= docker
PYTHON ?= python3
PYTEST_ARGS ?= -q
GPURUN ?= /usr/local/graft/bin/gpurun
export PYTHONPATH := $(CURDIR)

.PHONY: all
all: build

##@ General

.PHONY: help
help: ## Display this help.
	@awk 'BEGIN {FS = ":.*##"; printf "\nUsage:\n  make \033[36m<target>\033[0m\n"} /^[a-zA-Z_0-9-]+:.*?##/ { printf "  \033[36m%-18s\033[0m %s\n", $$1, $$2 } /^##@/ { printf "\n\033[1m%s\033[0m\n", substr($$0, 5) } ' $(MAKEFILE_LIST)

##@ Development

.PHONY: manifests
manifests: ## Regenerate the CRD (charts/ + deploy/kustomize/crd) and the manager ClusterRole from the Python types.
	$(PYTHON) -m cron_operator_amd.api.v1alpha1.crd
	$(PYTHON) -m cron_operator_amd.controller.rbac

.PHONY: generate
generate: manifests ## Alias: there is no deepcopy codegen (objects are plain dicts + dataclasses).

.PHONY: fmt
fmt: ## Normalise whitespace (trailing spaces, final newline) in Python sources.
	$(PYTHON) scripts/lint.py --fix

.PHONY: vet
vet: ## Byte-compile every module and import the package (the `go vet` analog).
	$(PYTHON) -m compileall -q cron_operator_amd tests scripts bench.py __graft_entry__.py
	$(PYTHON) -c "import cron_operator_amd.cmd.main, cron_operator_amd.controller.reconciler"

.PHONY: lint
lint: vet ## Static checks: unused imports/names, line length, whitespace (stdlib only).
	$(PYTHON) scripts/lint.py

.PHONY: sanitize
sanitize: ## ASan + UBSan build of the C++ extensions, fuzzed and property-driven (host code only).
	$(PYTHON) scripts/sanitize.py

.PHONY: test
test: build ## CPU test tiers: unit, envtest-analog, manager integration, e2e processes, chart/manifests.
	$(PYTHON) -m pytest tests/ -m "not gpu" $(PYTEST_ARGS)

.PHONY: test-e2e
test-e2e: build ## Process-level e2e (operator binary against an HTTP apiserver process).
	$(PYTHON) -m pytest tests/test_e2e.py $(PYTEST_ARGS)

.PHONY: test-gpu
test-gpu: build ## GPU tier on an MI355X (scheduled payload on cuda:0, RCCL DDP, native code loaded).
	$(PYTHON) -m pytest tests/ -m gpu -x $(PYTEST_ARGS)

.PHONY: test-gpu-remote
test-gpu-remote: build ## Run the GPU tier + bench + smoke on a gpurun MI355X box.
	$(GPURUN) --timeout 1200 -- 'STEPS="tests bench rocprof" bash scripts/gpu_run.sh'

.PHONY: sanity-check
sanity-check: manifests ## CI sanity: generated files must be committed (no diff after `make manifests`).
	git diff --exit-code -- charts deploy

##@ Build

.PHONY: build
build: ## Compile the native components in-tree (cron engine, JSON-tree ops).
	$(PYTHON) -m cron_operator_amd.ops.build

.PHONY: run
run: build ## Run the operator against the current kubeconfig (out of cluster).
	$(PYTHON) -m cron_operator_amd start --metrics-bind-address=:8080 --metrics-secure=false

.PHONY: run-fake
run-fake: build ## Fake apiserver + fake training-operator on :6443, kubeconfig in ./bin/kubeconfig.
	mkdir -p bin
	$(PYTHON) -m cron_operator_amd fake-apiserver --port 6443 --kubeconfig-out bin/kubeconfig --training-operator

.PHONY: bench
bench: build ## Headline benchmark (1000 Crons, `* * * * *`, historyLimit=10) -> one JSON line.
	$(PYTHON) bench.py

.PHONY: bench-reference
bench-reference: build ## Same benchmark with the reference algorithm (BASELINE.md denominator).
	$(PYTHON) bench.py --mode reference --steps 3 --warmup 1

.PHONY: bench-baseline-configs
bench-baseline-configs: build ## All five BASELINE.json configs in both modes, with their invariants checked.
	$(PYTHON) scripts/baseline_configs.py --out baseline_configs.json

.PHONY: bench-scale
bench-scale: build ## Scaling curve over 1/10/100/1000 Crons (BASELINE.json configs).
	$(PYTHON) scripts/bench_scale.py

.PHONY: docker-build
docker-build: ## Build the operator image.
	$(CONTAINER_TOOL) build -t $(IMG) .

.PHONY: docker-push
docker-push: ## Push the operator image.
	$(CONTAINER_TOOL) push $(IMG)

.PHONY: docker-build-payload
docker-build-payload: ## Build the MI355X payload image the examples/mi355x Crons run.
	$(CONTAINER_TOOL) build -f Dockerfile.payload --build-arg ROCM_PYTORCH_IMAGE=$(ROCM_PYTORCH_IMAGE) -t $(PAYLOAD_IMG) .

.PHONY: docker-push-payload
docker-push-payload: ## Push the MI355X payload image.
	$(CONTAINER_TOOL) push $(PAYLOAD_IMG)

PLATFORMS ?= linux/amd64,linux/arm64
.PHONY: docker-buildx
docker-buildx: ## Multi-arch build and push.
	- $(CONTAINER_TOOL) buildx create --name cron-operator-builder
	$(CONTAINER_TOOL) buildx use cron-operator-builder
	- $(CONTAINER_TOOL) buildx build --push --platform=$(PLATFORMS) --tag $(IMG) .
	- $(CONTAINER_TOOL) buildx rm cron-operator-builder

.PHONY: build-installer
build-installer: manifests ## Render deploy/kustomize/default into dist/install.yaml.
	$(PYTHON) -m cron_operator_amd kustomize deploy/kustomize/default -o dist/install.yaml

.PHONY: build-installer-certs
build-installer-certs: manifests ## Render deploy/kustomize/default with cert-manager metrics TLS, ServiceMonitor and network policy into dist/install-certs.yaml.
	$(PYTHON) -m cron_operator_amd kustomize --enable-optional deploy/kustomize/default -o dist/install-certs.yaml

##@ Helm

.PHONY: helm-unittest
helm-unittest: ## Run the chart's helm-unittest suites (charts/cron-operator/tests) + chart render tests.
	$(PYTHON) -m cron_operator_amd.utils.helmunittest
	$(PYTHON) -m pytest tests/test_helm_chart.py $(PYTEST_ARGS)

.PHONY: helm-template
helm-template: ## Render the chart with default values.
	$(PYTHON) -m cron_operator_amd helm-template charts/cron-operator

.PHONY: helm-docs
helm-docs: ## Regenerate the values table in charts/cron-operator/README.md.
	$(PYTHON) scripts/helm_docs.py

.PHONY: helm-upgrade
helm-upgrade: ## Install/upgrade the chart into the current cluster (needs helm).
	helm upgrade cron-operator charts/cron-operator --install --namespace cron-operator --create-namespace \
		--set image.registry=$(IMG_REGISTRY) --set image.repository=$(IMG_REPOSITORY) --set image.tag=$(IMG_TAG)

.PHONY: helm-uninstall
helm-uninstall: ## Uninstall the chart.
	helm uninstall cron-operator --namespace cron-operator

##@ kind (local cluster; needs kind + kubectl + helm)

KIND_CLUSTER ?= cron-operator
KIND_K8S_VERSION ?= v1.34.0

.PHONY: kind-create-cluster
kind-create-cluster: ## Create a kind cluster for e2e runs against a real apiserver.
	kind create cluster --name $(KIND_CLUSTER) --image kindest/node:$(KIND_K8S_VERSION)

.PHONY: kind-load-image
kind-load-image: docker-build ## Load the operator image into the kind cluster.
	kind load docker-image $(IMG) --name $(KIND_CLUSTER)

.PHONY: test-e2e-cluster
test-e2e-cluster: kind-load-image deploy ## Real-cluster e2e (test/e2e analog): pod Running/Ready, authn'd /metrics via a curl pod, a Cron fires.
	kubectl -n cron-operator-system rollout status deploy/cron-operator-controller-manager --timeout=180s
	E2E_CLUSTER=1 $(PYTHON) -m pytest tests/test_e2e_cluster.py -v -p no:cacheprovider

.PHONY: kind-delete-cluster
kind-delete-cluster: ## Delete the kind cluster.
	kind delete cluster --name $(KIND_CLUSTER)

.PHONY: test-e2e-kind
test-e2e-kind: kind-load-image helm-upgrade ## Real-cluster smoke: operator Running, a Cron fires (test/e2e analog).
	kubectl -n cron-operator rollout status deploy/cron-operator --timeout=180s
	kubectl apply -f examples/v1alpha1/cron/cron-pod.yaml
	kubectl wait --for=jsonpath='{.status.lastScheduleTime}' cron/heartbeat-pod --timeout=120s

##@ Deployment

ignore-not-found ?= false

.PHONY: install
install: manifests ## Install the CRD into the cluster in ~/.kube/config.
	$(PYTHON) -m cron_operator_amd kustomize deploy/kustomize/crd | kubectl apply -f -

.PHONY: uninstall
uninstall: ## Remove the CRD.
	$(PYTHON) -m cron_operator_amd kustomize deploy/kustomize/crd | kubectl delete --ignore-not-found=$(ignore-not-found) -f -

.PHONY: deploy
deploy: manifests ## Deploy the operator (kustomize default overlay) with IMG.
	$(PYTHON) -m cron_operator_amd kustomize deploy/kustomize/default | sed 's#docker.io/cron-operator-amd/cron-operator:[^ ]*#$(IMG)#' | kubectl apply -f -

.PHONY: undeploy
undeploy: ## Remove the operator.
	$(PYTHON) -m cron_operator_amd kustomize deploy/kustomize/default | kubectl delete --ignore-not-found=$(ignore-not-found) -f -

.PHONY: clean
clean: ## Remove built native libraries and dist/.
	rm -rf dist bin cron_operator_amd/ops/*.so
