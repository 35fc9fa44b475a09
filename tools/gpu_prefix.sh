# sr_plan_first's first prefix batch: end-to-end tick per SR_PREFIX_BATCH, C3 and C4
cd "$GRAFT_REPO_ROOT" || exit 2
out=gpurun_out/${TAG:-prefix}
mkdir -p $out
for cfg in ${CFGS:-3 4 2 5 1}; do
  for b in 64 32 16 8; do
    steps=50; [ $cfg = 4 ] && steps=20
    SR_PREFIX_BATCH=$b timeout -k 10 300 python bench.py --config $cfg --steps $steps --warmup 5 --no-cpu-baseline \
      > $out/c${cfg}_b$b.log 2>&1 || exit $?
    tail -1 $out/c${cfg}_b$b.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());e=d['end_to_end_tick']
print('C$cfg batch $b e2e median %.4f min %.4f batches %s enc %.4f full %.3f' % (e['median_ms'],e['min_ms'],e['prefix_batches'],e['encode_ms_last_batch'],e['full_tick_median_ms']))"
  done
done
