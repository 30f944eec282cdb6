# Operator image (reference Dockerfile:1-40 builds a static Go binary on distroless; this one runs
# the Python controller on a slim base as the same non-root UID).
FROM python:3.10-slim
RUN pip install --no-cache-dir httpx pyyaml prometheus_client
WORKDIR /opt/omx
COPY ollama_operator_amd/__init__.py ./ollama_operator_amd/__init__.py
COPY ollama_operator_amd/operator ./ollama_operator_amd/operator
USER 65532:65532
ENTRYPOINT ["python3", "-m", "ollama_operator_amd.operator"]
