#!/bin/bash
# Tick-only kernel (k_tick_bench): timing plus one PMC pass of issue counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/tick_bench.py > gpurun_out/tick.log 2>&1 || { tail -3 gpurun_out/tick.log; exit 1; }
grep '^{' gpurun_out/tick.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU \
    --kernel-trace --output-format csv -d gpurun_out/tick_pmc -o run -- python3 tools/tick_bench.py > gpurun_out/tick_pmc.log 2>&1 || { tail -3 gpurun_out/tick_pmc.log; exit 1; }
python3 - <<'PY'
import csv, collections
d = collections.defaultdict(dict)
for r in csv.DictReader(open('gpurun_out/tick_pmc/run_counter_collection.csv')):
    if 'k_tick_bench' in r['Kernel_Name']:
        d[r['Dispatch_Id']][r['Counter_Name']] = float(r['Counter_Value'])
last = d[max(d, key=int)]
print({k: v for k, v in last.items()})
w = last['SQ_WAVES']
print('valu/wave', last['SQ_INSTS_VALU'] / w, 'salu/wave', last['SQ_INSTS_SALU'] / w,
      'active_valu_frac', last['SQ_ACTIVE_INST_VALU'] / last['SQ_WAVE_CYCLES'], 'wait_any_frac', last['SQ_WAIT_ANY'] / last['SQ_WAVE_CYCLES'])
PY
