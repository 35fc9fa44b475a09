# SQ / SQC counters of the C3 tick (instruction cache, wait and issue cycles), two passes
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
out="$R/gpurun_out/${TAG:-sqpmc}"
mkdir -p "$out"
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH \
  --kernel-trace -d "$out/p1" -o run --output-format csv -- \
  python3 "$R/bench.py" --config ${CFG:-3} --steps 20 --warmup 2 --no-cpu-baseline --e2e-reps 1 > "$out/p1.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
  SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU --kernel-trace -d "$out/p2" -o run --output-format csv -- \
  python3 "$R/bench.py" --config ${CFG:-3} --steps 20 --warmup 2 --no-cpu-baseline --e2e-reps 1 > "$out/p2.log" 2>&1 || exit $?
cd "$R" && python3 tools/sq_summary.py "$out"
