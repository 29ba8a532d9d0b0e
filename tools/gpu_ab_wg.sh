cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
for lib in product exp_build/libsalp_wg128.so; do
  l=$lib; [ "$lib" = product ] && l=""
  SALP_LIB=$l N="32768 65536" K=32 timeout -k 10 200 python tools/collect_bench.py > gpurun_out/abwg_c.log 2>&1 || { tail -5 gpurun_out/abwg_c.log; exit 1; }
  echo "$lib"; cat gpurun_out/abwg_c.log | grep n_envs
  SALP_LIB=$l timeout -k 10 200 python bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-parity-check > gpurun_out/abwg_b.log 2>&1 || { tail -5 gpurun_out/abwg_b.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abwg_b.log').read().strip().splitlines()[-1]);print('$lib', round(d['value']/1e6,3), d['kernel_ms_per_launch'], d.get('ppo',{}).get('value'))"
done; done
