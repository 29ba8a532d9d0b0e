cd "${GRAFT_REPO_ROOT}" || exit 1
for r in 1 2; do for lib in exp_build/libsalp_rep1.so product; do
  l=$lib; [ "$lib" = product ] && l=""
  SALP_LIB=$l N=65536 K=32 timeout -k 10 200 python tools/collect_bench.py 2>/dev/null | grep n_envs | sed "s|^|$lib |" >> gpurun_out/r4rep_c65.txt || exit 1
done; done
