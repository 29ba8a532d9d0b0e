#!/bin/bash
# Host-ASan/UBSan build of the C ABI driven end to end on the GPU (host code
# instrumented only: -Xarch_host; no GPU sanitizer).  tools/sanitize/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 make -s -C tools/sanitize gpu > gpurun_out/sanitize_gpu.log 2>&1
rc=$?
grep -v "^\s*#" gpurun_out/sanitize_gpu.log | tail -n 8
exit $rc
