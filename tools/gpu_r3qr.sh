#!/bin/bash
# The SQ-counter probe of the bf16 3x3 kernels, then the bf16 stream-switch A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
bash tools/gpu_r3r.sh && bash tools/gpu_r3q.sh
