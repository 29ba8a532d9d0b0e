set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for c in 64 96 128; do timeout -k 10 120 python bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-lockstep --chunk $c > gpurun_out/b_new_$c.log 2>&1 || exit 1; python -c "import json;d=json.loads(open('gpurun_out/b_new_$c.log').read().strip().splitlines()[-1]);print('new',$c,d['value']/1e6,d['kernel_ms_per_launch'])"; done
SALP_ROLLOUT_V1=1 timeout -k 10 120 python bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-lockstep --chunk 128 > gpurun_out/b_v1.log 2>&1 || exit 1
python -c "import json;d=json.loads(open('gpurun_out/b_v1.log').read().strip().splitlines()[-1]);print('v1',128,d['value']/1e6,d['kernel_ms_per_launch'])"
