#!/bin/bash
# Event-timed K2 duration vs rocprofv3's kernel trace, for --event-every 1 and 16.
cd "$GRAFT_REPO_ROOT" || exit 2
T=${1:-evcheck}; out=gpurun_out/$T; mkdir -p $out
for ev in 16 1 16 1; do
  timeout -k 10 200 python bench.py --config 3 --steps 400 --warmup 20 --no-cpu-baseline --e2e-reps 0 --event-every $ev \
    > $out/bench_ev$ev.log 2>&1 || exit $?
  python -c "
import json,sys; d=json.loads(open('$out/bench_ev$ev.log').read().strip().splitlines()[-1])
print('event-every $ev: ms/step %.4f  calib K2 %.4f  timed K2 %.5f' % (d['ms_per_step'], d['kernels_ms']['k2_placement'], d['roofline']['kernel_ms']))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --config 3 --steps 400 --warmup 20 --no-cpu-baseline --e2e-reps 0 > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1 || exit $?
f=$(find "$GRAFT_REPO_ROOT/$out/prof" -name '*kernel_stats.csv' | head -1); cut -c1-160 "$f"
