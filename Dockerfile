# Operator image.  Reference: Dockerfile:1-28 (static Go binary on debian-12-slim,
# USER 65534).  Here: stage 1 compiles the native C++ components (cron engine,
# JSON-tree ops, HTTP framing) against the image's CPython; stage 2 carries only
# the package, its runtime deps and the built .so files.  Zones: the tzdata wheel
# (Go's embedded time/tzdata) plus the OS zoneinfo tree, searched in Go's order.  No GPU stack: the operator is
# control plane; the MI355X workloads it schedules use their own ROCm images.
ARG PYTHON_IMAGE=python:3.10-slim-bookworm

FROM ${PYTHON_IMAGE} AS builder
RUN apt-get update && apt-get install -y --no-install-recommends g++ && rm -rf /var/lib/apt/lists/*
WORKDIR /workspace
COPY pyproject.toml README.md ./
COPY cron_operator_amd ./cron_operator_amd
RUN python -m cron_operator_amd.ops.build --force \
 && pip install --no-cache-dir --prefix=/install aiohttp PyYAML tzdata \
 && find cron_operator_amd -name '__pycache__' -prune -exec rm -rf {} +

FROM ${PYTHON_IMAGE}
RUN apt-get update && apt-get install -y --no-install-recommends tzdata && rm -rf /var/lib/apt/lists/*
WORKDIR /app
COPY --from=builder /install /usr/local
COPY --from=builder /workspace/cron_operator_amd ./cron_operator_amd
ENV PYTHONUNBUFFERED=1 PYTHONDONTWRITEBYTECODE=1 CRON_OPERATOR_ENGINE=native
USER 65534:65534
ENTRYPOINT ["python", "-m", "cron_operator_amd"]
CMD ["start"]
