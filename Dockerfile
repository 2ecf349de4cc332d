# MI355X (gfx950) development image: ROCm PyTorch + this framework's native extension.
#
# Pinned to the stack this framework is built and measured on (every number under profiles/):
# ROCm 7.2.0, PyTorch 2.10.0 built for ROCm 7.0, Python 3.10.  Override BASE_IMAGE with the
# matching tag (or digest, rocm/pytorch@sha256:...) of your registry mirror; the version check
# below refuses an image whose stack differs.
ARG BASE_IMAGE=rocm/pytorch:rocm7.2_ubuntu22.04_py3.10_pytorch_release_2.10.0
FROM ${BASE_IMAGE}

ARG EXPECT_TORCH=2.10.0
ARG EXPECT_ROCM=7.2.0
RUN python3 -c "import torch, sys; v = torch.__version__.split('+')[0]; \
sys.exit(0 if v == '${EXPECT_TORCH}' and torch.version.hip else 'torch ' + torch.__version__ + ' != ${EXPECT_TORCH} (ROCm build)')" && \
    grep -q "^${EXPECT_ROCM}" /opt/rocm/.info/version || (echo "ROCm $(cat /opt/rocm/.info/version) != ${EXPECT_ROCM}" && false)

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
