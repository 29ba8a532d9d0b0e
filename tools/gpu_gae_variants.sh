for v in ${GAE_VARIANTS:-product gae8 gae32 gae64}; do
  lib=""; [ "$v" != product ] && lib="exp_build/libsalp_$v.so"
  SALP_LIB=$lib timeout -k 10 120 python tools/gae_bench.py 2>&1 | grep '^{' || exit 1
done
