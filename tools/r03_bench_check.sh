#!/bin/bash
# the default bench line twice + its rocprof kernel stats (the roofline kernel's per-dispatch mean),
# then BASELINE configs 3-5
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r03c}
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-exact > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err || { tail -5 gpurun_out/${T}_bench$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_bench$i.json')); r=d['roofline']; print(d['value'], r['launch_us'], r.get('event_pair_us'), r['frac'], d['lookup_b8']['frac'], d['iteration']['iteration_us'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python bench.py --no-cpu-baseline --no-fp32-exact > gpurun_out/${T}_bench_under_rocprof.json 2> gpurun_out/${T}_rocprof.err || exit 1
python -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_$T/run_kernel_stats.csv')):
    if 'lookup_conv_kernel' in r['Name']: print('rocprof lookup_conv', r['Calls'], float(r['AverageNs'])/1e3)
"
./tools/config_sweep.sh $T
