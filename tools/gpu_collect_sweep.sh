#!/bin/bash
# salp_collect chunk x steady-budget sweep (tools/collect_bench.py, K env-steps
# per env per call); one line per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for q in ${QS:-400 480}; do
  for c in ${CHUNKS:-256 384 512}; do
    SALP_STEADY_Q8=$q SALP_COLLECT_CHUNK=$c timeout -k 10 200 python -u tools/collect_bench.py > gpurun_out/cs.jsonl 2>/dev/null || exit 1
    python -c "import json;[print('q',$q,'chunk',$c,d['n_envs'],d['collect_0'],d['collect_1'],d['rollout_cap_1'],d['step_random_1']) for d in map(json.loads,open('gpurun_out/cs.jsonl'))]" | tee -a gpurun_out/collect_sweep.txt
  done
done
