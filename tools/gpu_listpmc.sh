cd /tmp && export TMPDIR=/tmp
mkdir -p "$GRAFT_REPO_ROOT/gpurun_out/pmc"
timeout -k 10 120 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/pmc/list.txt" 2>&1
grep -oE "(SQC_[A-Z_0-9]+|SQ_WAIT[A-Z_0-9]*|SQ_INSTS_[A-Z_0-9]+|SQ_WAVE_CYCLES|SQ_BUSY_CYCLES|SQ_INST_CYCLES_[A-Z_0-9]+|SQ_IFETCH[A-Z_0-9]*|SQ_ACTIVE_INST_[A-Z_0-9]+)" "$GRAFT_REPO_ROOT/gpurun_out/pmc/list.txt" | sort -u | tr '\n' ' '
