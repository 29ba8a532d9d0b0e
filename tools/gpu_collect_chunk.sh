#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
set -o pipefail
for c in ${CHUNKS:-128 192 256 384}; do
  SALP_COLLECT_CHUNK=$c timeout -k 10 200 python -u tools/collect_bench.py > gpurun_out/cc_$c.jsonl 2>/dev/null || exit 1
  python -c "import json;[print('chunk',$c,d['n_envs'],d['collect_0'],d['collect_1'],d['rollout_cap_1']) for d in map(json.loads,open('gpurun_out/cc_$c.jsonl'))]"
done
