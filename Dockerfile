# Runtime/dev image recipe: ROCm 7 + PyTorch-ROCm base, then the in-tree native build.
# (The reference ships a Dockerfile for its comet worker; this one serves the same role:
#  `docker run --device=/dev/kfd --device=/dev/dri moose-amd comet --identity alice ...`.)
FROM rocm/pytorch:latest
ENV PYTORCH_ROCM_ARCH=gfx950 HSA_ENABLE_IPC_MODE_LEGACY=0
WORKDIR /opt/moose_amd
COPY . .
RUN python -c "import __graft_entry__ as g; g.build()" && pip install --no-deps -e .
CMD ["comet", "--help"]
