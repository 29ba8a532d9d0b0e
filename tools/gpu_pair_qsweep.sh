cd $GRAFT_REPO_ROOT
for q in 300 380 480; do for ch in 256 384 512; do
  SALP_STEADY_Q8=$q SALP_COLLECT_CHUNK=$ch SALP_ROLLOUT_KERNEL=1 N="32768" K=32 timeout -k 10 100 python tools/collect_bench.py 2>/dev/null | grep n_envs | sed "s/^/q=$q ch=$ch /" >> gpurun_out/r4h_qsweep.txt || exit 1
done; done
