# MI355X (gfx950) development image: ROCm PyTorch + this framework's native extension.
FROM rocm/pytorch:latest

RUN apt-get update && apt-get install -y --no-install-recommends git tmux && \
    apt-get clean && rm -rf /var/lib/apt/lists/* && \
    git config --global --add safe.directory /workspace

COPY requirements.txt /tmp/requirements.txt
RUN pip install -r /tmp/requirements.txt

ENV PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    OMP_NUM_THREADS=1
WORKDIR /workspace
# Build the gfx950 kernels in-tree on first use:  python csrc/build.py
