#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O2 -o /tmp/probe tests/native/probe_fragments.hip 2>/dev/null
timeout -k 10 120 /tmp/probe > gpurun_out/probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/probe.log
