#!/bin/bash
# BASELINE config 5 (PPO, 32 768 envs): a 24-iteration learning trend at
# n_steps 32, then the timed run at the reference's n_steps 2048
# (src/train_robot_recurrent_ppo.py:91), and a rocprofv3 kernel summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r2f}
timeout -k 10 300 python -u tools/bench_ppo.py --n-steps 32 --iters 2 --trend-iters 24 > gpurun_out/${TAG}_ppo32.json 2> gpurun_out/${TAG}_ppo32.err || { tail -5 gpurun_out/${TAG}_ppo32.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_ppo32.json').read().strip().splitlines()[-1]);print('n_steps 32:', round(d['value']/1e6,3), d['timing_s'], [ (r['iteration'], round(r['ep_return_mean'] or 0,1), r['diverged_envs'], round(r['vf_loss'],2)) for r in d['trend']])"
timeout -k 10 400 python -u tools/bench_ppo.py --n-steps 2048 --iters 1 > gpurun_out/${TAG}_ppo2048.json 2> gpurun_out/${TAG}_ppo2048.err || { tail -5 gpurun_out/${TAG}_ppo2048.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_ppo2048.json').read().strip().splitlines()[-1]);print('n_steps 2048:', round(d['value']/1e6,3), d['timing_s'], d['losses'], d['diverged_envs_reset'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_ppo_prof -o run -- python3 tools/bench_ppo.py --n-steps 32 --iters 1 > gpurun_out/${TAG}_ppo_prof.log 2>&1 || { tail -5 gpurun_out/${TAG}_ppo_prof.log; exit 1; }
head -12 gpurun_out/${TAG}_ppo_prof/run_kernel_stats.csv | cut -c1-160
