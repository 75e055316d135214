#!/bin/bash
# SQ counter passes over the sort workload (downsweep stall study), one
# rocprofv3 --pmc run per counter set.  Output: gpurun_out/sortpmc/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O="$R/gpurun_out/sortpmc"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for PS in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PS -d "$O/p$i" -o run -f csv -- python3 "$R/bench.py" --workload ${WL:-sort} --steps 3 --warmup 1 --no-cpu-baseline > "$O/p$i.log" 2>&1 || exit 1
  echo "done p$i" >> "$O/progress.log"
done
