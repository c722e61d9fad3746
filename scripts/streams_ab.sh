#!/bin/bash
# streams_ab.sh [TAG]: the headline with --streams 4, 2 and 1 alternating (twice each, side
# lines off), the full bench line, and a rocprofv3 kernel trace of the headline; the trace
# is split into overlapped and back-to-back launches by scripts/stream_regions.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-streams}; mkdir -p $O
SIDE="--dense-steps 0 --band-steps 0 --sample-traj 0 --config5 0 --config4 0 --cache-resident 0 --host-line 0 --node-line 0 --uniform-large-m 0 --config2 0 --cpu-seconds 0"
for s in 4 2 1 4 2 1; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 5 --streams $s $SIDE >> $O/ab_streams.jsonl 2>> $O/ab.err || exit 1
done
timeout -k 10 400 python bench.py --steps 50 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 $SIDE > $O/prof_bench.json 2> $O/prof.err || exit 1
python3 -c "
import json
for l in open('$O/ab_streams.jsonl'):
    d=json.loads(l); r=d['roofline']; print(d['config']['streams_per_device'], round(d['value']/1e9,4), round(d['ms_per_step']*1e3,2), round(r['launch_ms']*1e3,2), round(r['frac'],4), round(r['pipelined']['frac'],4))
"
python3 scripts/stream_regions.py $O/prof/run_kernel_trace.csv > $O/stream_regions.json
cut -c1-300 $O/bench.json
