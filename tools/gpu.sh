#!/bin/bash
# One parametrised GPU session (replaces the per-round gpu_r*.sh one-offs).
#
#   tools/gpu.sh OUT STEP [STEP ...]          (run from the repo root, under gpurun)
#
# Output goes to gpurun_out/OUT/ (progress.log + one log per step).  Each STEP
# is one quoted string; every GPU step runs under its own time limit and the
# first failure ends the session (no retries):
#   tests [PYTEST ARGS]             the -m gpu suite (-x, per-test 120 s timeout); ARGS
#                                   (test files, -k EXPR) replace the default `tests`
#   smoke                           __graft_entry__.smoke()
#   bench NAME [BENCH ARGS]         python bench.py ARGS > NAME.json (the JSON line) + NAME.log
#   benv NAME K=V[,K=V] [BENCH ARGS]  the same with environment variables set (e.g.
#                                   LHPC_LIB_PATH=libhpc_amd/_abx/X/liblhpc.so for an A/B build)
#   stats NAME [BENCH ARGS]         the same under rocprofv3 --kernel-trace --stats (NAME/ dir)
#   senv NAME K=PATH[,K=PATH] [BENCH ARGS]  stats with K=$REPO/PATH exported first (A/B library paths;
#                                   - for none: the same step on the default library)
#   pmc NAME COUNTERS [BENCH ARGS]  one rocprofv3 --pmc pass (COUNTERS comma-separated)
#   py NAME SCRIPT [ARGS]           python SCRIPT ARGS > NAME.log (tools/*.py probes)
#   spy NAME K=V[,K=V] SCRIPT [ARGS]  the same under rocprofv3 --kernel-trace --stats, with K=V
#                                   exported (a V naming libhpc_amd/… is made absolute; - for none)
#   dist NAME NPROC [BENCH ARGS]    bench.py under torch.distributed.run (env passed through)
# Limits: tests 1100 s, stats/bench/py/dist 600 s, pmc 240 s (SIGKILL).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
O="$R/gpurun_out/$1"; shift; mkdir -p "$O"
export TMPDIR=/tmp
log() { echo "$(date +%T) $*" >> "$O/progress.log"; }
run() {  # run NAME SECS SIGNAL CMD...
  local name=$1 secs=$2 sig=$3; shift 3
  log "start $name"
  timeout -s "$sig" -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  log "end $name rc=$rc"
  return $rc
}
for S in "$@"; do
  read -ra A <<< "$S"
  kind=${A[0]}
  case $kind in
    tests)
      T=("${A[@]:1}"); [ ${#T[@]} -eq 0 ] && T=(tests)
      run pytest_gpu 1100 TERM python -u -m pytest "${T[@]}" -m gpu -x -v -p no:cacheprovider --timeout 120 \
        --timeout-method thread || exit 1 ;;
    smoke)
      run smoke 300 TERM python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench)
      run "${A[1]}" 600 TERM python bench.py "${A[@]:2}" || exit 1
      grep '^{' "$O/${A[1]}.log" | tail -1 > "$O/${A[1]}.json" ;;
    benv)
      IFS=',' read -ra KV <<< "${A[2]}"
      run "${A[1]}" 600 TERM env "${KV[@]}" python bench.py "${A[@]:3}" || exit 1
      grep '^{' "$O/${A[1]}.log" | tail -1 > "$O/${A[1]}.json" ;;
    stats)
      (cd /tmp && run "${A[1]}" 600 TERM rocprofv3 --kernel-trace --stats -d "$O/${A[1]}" -o run -f csv -- \
        python3 "$R/bench.py" "${A[@]:2}") || exit 1
      grep '^{' "$O/${A[1]}.log" | tail -1 > "$O/${A[1]}.json" ;;
    senv)
      IFS=',' read -ra KV <<< "${A[2]}"
      (for kv in "${KV[@]}"; do [ "$kv" = "-" ] && continue; export "${kv%%=*}=$R/${kv#*=}"; done
       cd /tmp && run "${A[1]}" 600 TERM rocprofv3 --kernel-trace --stats -d "$O/${A[1]}" -o run -f csv -- \
        python3 "$R/bench.py" "${A[@]:3}") || exit 1
      grep '^{' "$O/${A[1]}.log" | tail -1 > "$O/${A[1]}.json" ;;
    pmc)
      (cd /tmp && run "${A[1]}" 240 KILL rocprofv3 --pmc ${A[2]//,/ } -d "$O/${A[1]}" -o run -f csv -- \
        python3 "$R/bench.py" "${A[@]:3}") || exit 1 ;;
    py)
      run "${A[1]}" 600 TERM python -u "${A[@]:2}" || exit 1 ;;
    spy)
      IFS=',' read -ra KV <<< "${A[2]}"
      (for kv in "${KV[@]}"; do [ "$kv" = "-" ] && continue; v=${kv#*=}; [[ $v == libhpc_amd/* ]] && v=$R/$v
         export "${kv%%=*}=$v"; done
       cd /tmp && run "${A[1]}" 600 TERM rocprofv3 --kernel-trace --stats -d "$O/${A[1]}" -o run -f csv -- \
        python3 -u "$R/${A[3]}" "${A[@]:4}") || exit 1 ;;
    dist)
      run "${A[1]}" 600 TERM python -m torch.distributed.run --nnodes=1 --nproc-per-node "${A[2]}" \
        --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) bench.py "${A[@]:3}" || exit 1 ;;
    *)
      log "unknown step $kind"; exit 2 ;;
  esac
done
log done
exit 0
