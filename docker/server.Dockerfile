# MI355X inference server image: replaces `ollama/ollama` in the pods the operator launches
# (reference pkg/model/pod.go:10-12). Entrypoint `ollama` provides `serve` and `pull`.
ARG BASE=rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.7.1
FROM ${BASE}
ENV PYTORCH_ROCM_ARCH=gfx950 OMX_ARCH=gfx950 OLLAMA_HOST=0.0.0.0 OLLAMA_MODELS=/root/.ollama/models
WORKDIR /opt/omx
RUN pip install --no-cache-dir fastapi uvicorn httpx pyyaml prometheus_client regex pybind11
COPY build_native.py ./
COPY csrc ./csrc
COPY ollama_operator_amd ./ollama_operator_amd
COPY bin ./bin
RUN python3 build_native.py && ln -s /opt/omx/bin/ollama /usr/local/bin/ollama
EXPOSE 11434
ENTRYPOINT ["ollama"]
CMD ["serve"]
