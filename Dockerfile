# dmcp service image on ROCm (the base image carries PyTorch-ROCm, hipcc and
# the ROCm runtime; the GPU is only used by ENRICH_BACKEND=local).
# Parity: the reference's Dockerfile (eclipse-temurin:21-jre + release JAR).
ARG BASE=rocm/pytorch:latest
FROM ${BASE}

RUN apt-get update && apt-get install -y --no-install-recommends git ca-certificates \
    && rm -rf /var/lib/apt/lists/*
WORKDIR /opt/dmcp
COPY dmcp/ dmcp/
COPY native/ native/
COPY bench.py bench_enrich.py __graft_entry__.py pytest.ini ./
COPY scripts/ scripts/
RUN pip install --no-cache-dir fastapi uvicorn pybind11 pyyaml safetensors \
    && PYTORCH_ROCM_ARCH=gfx950 python -m dmcp.buildtools

ENV DMCP_DB_PATH=/data/dmcp.db \
    GIT_CLONE_BASE_PATH=/tmp/domain-mcp-repos \
    SERVER_HOST=0.0.0.0 \
    SERVER_PORT=8080
VOLUME ["/data"]
EXPOSE 8080
ENTRYPOINT ["python", "-m", "dmcp"]
CMD ["serve", "--host", "0.0.0.0"]
