#!/bin/bash
# One validation pass of a kept change set: the GPU suite,
# the default bench line, its rocprofv3 kernel statistics, the PMC passes of
# the headline kernel and of config 5's collection kernel (through
# tools/collect_pmc_probe.py), and the per-env step path's latency.  Then, here:
#   python tools/pmc_summary.py TAG
#   python tools/pmc_summary.py TAGc --kernel 'k_rollout_split<true>' --symbol k_rollout_splitILb1EE \
#       --config-json '{"n_envs": 32768, "n_steps": 256}' --suffix pmc_collect_summary \
#       --workload-json gpurun_out/TAG_collect_probe.json
# TAG names the outputs under gpurun_out/ (the collection's PMC passes: TAGc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-final}
set -o pipefail
echo "== pytest $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "gpurun_out/${TAG}_pytest_gpu.txt" 2>&1 || { tail -30 "gpurun_out/${TAG}_pytest_gpu.txt"; exit 1; }
tail -1 "gpurun_out/${TAG}_pytest_gpu.txt"
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/${TAG}_smoke.txt" 2>&1 \
    || { tail -30 "gpurun_out/${TAG}_smoke.txt"; exit 1; }
echo "== bench $(date +%T)"
timeout -k 10 600 python bench.py > "gpurun_out/${TAG}_bench.json" 2> "gpurun_out/${TAG}_bench.err" || exit 1
tail -c 300 "gpurun_out/${TAG}_bench.json"
echo "== rocprofv3 stats $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${TAG}_prof" -o run \
    -- python3 bench.py > "gpurun_out/${TAG}_prof_bench.json" 2> "gpurun_out/${TAG}_prof.err" || exit 1
if [ "${SKIP_PMC:-0}" != 1 ]; then   # SKIP_PMC=1: both kernels' fingerprints unchanged since the last summaries
    echo "== pmc $(date +%T)"
    TAG=$TAG bash tools/gpu_pmc.sh || exit 1
    echo "== pmc collection $(date +%T)"
    timeout -k 10 300 python tools/collect_pmc_probe.py > "gpurun_out/${TAG}_collect_probe.json" 2>/dev/null || exit 1
    TAG=${TAG}c PROBE=1 bash tools/gpu_pmc_collect.sh || exit 1
fi
echo "== per-env step latency $(date +%T)"
timeout -k 10 300 python tools/step_latency.py > "gpurun_out/${TAG}_step_latency.json" 2>/dev/null || exit 1
timeout -k 10 300 python tools/host_path_bench.py > "gpurun_out/${TAG}_host_path.json" 2>/dev/null || exit 1
echo "== done $(date +%T)"
