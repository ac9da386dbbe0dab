#!/bin/bash
# One parameterised runner for the GPU box (through gpurun), replacing the
# per-experiment scripts of rounds 1-4.  Every GPU step has its own time limit
# and the steps are chained: the first failure ends the call.
#
#   bash tools/gpu_run.sh TAG check
#       every GPU test, smoke(), the headline at the driver's shape (20 / 5)
#   bash tools/gpu_run.sh TAG ab ROUNDS 'ENV_A' 'ENV_B' [CMD...]
#       alternate two environment settings ROUNDS times over CMD (default: the
#       headline, 10 steps / 3 warm-up); each run's first stdout line -> ab.txt
#   bash tools/gpu_run.sh TAG run SECONDS CMD...
#       one command under its own limit, stdout -> out.txt
#   bash tools/gpu_run.sh TAG prof SECONDS WINDOW_MS CMD...
#       rocprofv3 kernel trace of CMD, summarised on the box (tools/rocpd_summary.py,
#       last WINDOW_MS of the run) -> summary.md
#   bash tools/gpu_run.sh TAG pmc 'COUNTERS' CMD...
#       one rocprofv3 --pmc pass (kernel trace only; respect the per-block slot
#       limits), killed hard after 120 s
# Several modes chain with '+' in one call: e.g.
#   bash tools/gpu_run.sh r5a check + ab 2 'MCP_X=0' 'MCP_X=1'
set -o pipefail
export TMPDIR=/tmp
TAG=${1:?tag}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
BENCH=(python -u bench.py --steps 10 --warmup 3)
STEP=0

fail() { echo "$1 failed"; tail -30 "$2"; exit 1; }

run_check() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1 || fail "gpu tests" "$O/gpu_tests.log"
  tail -1 "$O/gpu_tests.log"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
    || fail smoke "$O/smoke.log"
  tail -1 "$O/smoke.log"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.log" \
    || fail bench "$O/bench.log"
  cut -c1-400 "$O/bench.json"
}

run_ab() {
  local rounds=$1 ea=$2 eb=$3
  shift 3
  local cmd=("$@")
  [ ${#cmd[@]} -eq 0 ] && cmd=("${BENCH[@]}")
  for r in $(seq 1 "$rounds"); do
    for v in a b; do
      local envs=$ea
      [ $v = b ] && envs=$eb
      local f="$O/ab_${STEP}_${r}_$v"
      env $envs timeout -k 10 400 "${cmd[@]}" > "$f.out" 2> "$f.log" || fail "ab $v round $r" "$f.log"
      echo "$v [$envs] $(head -1 "$f.out" | cut -c1-300)" | tee -a "$O/ab.txt"
    done
  done
}

run_one() {
  local secs=$1
  shift
  timeout -k 10 "$secs" "$@" > "$O/out_$STEP.txt" 2> "$O/out_$STEP.log" || fail "run" "$O/out_$STEP.log"
  tail -20 "$O/out_$STEP.txt"
}

run_prof() {
  local secs=$1 win=$2
  shift 2
  timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats -f rocpd -d /tmp/prof_$STEP -o run -- "$@" \
    > "$O/prof_$STEP.out" 2> "$O/prof_$STEP.log" || fail rocprof "$O/prof_$STEP.log"
  head -1 "$O/prof_$STEP.out" | cut -c1-300
  python tools/rocpd_summary.py /tmp/prof_$STEP/run_results.db "$win" > "$O/summary_$STEP.md" 2>&1 \
    || fail summary "$O/summary_$STEP.md"
  head -40 "$O/summary_$STEP.md"
}

run_pmc() {
  local counters=$1
  shift
  # the database stays on the box (a counter pass over a serving run exceeds
  # the 64 MiB copied back); the per-kernel summary comes back
  timeout -s KILL 120 rocprofv3 --pmc $counters -f rocpd -d "/tmp/pmc_$STEP" -o run -- "$@" \
    > "$O/pmc_$STEP.log" 2>&1 || fail "pmc pass" "$O/pmc_$STEP.log"
  python tools/pmc_summary.py --by-kernel "$(find /tmp/pmc_$STEP -name '*.db' | head -1)" \
    > "$O/pmc_$STEP.md" 2>&1 || fail "pmc summary" "$O/pmc_$STEP.md"
  echo "pmc pass $STEP done"
}

# split the arguments at '+' into modes
while [ $# -gt 0 ]; do
  args=()
  while [ $# -gt 0 ] && [ "$1" != "+" ]; do
    args+=("$1")
    shift
  done
  [ $# -gt 0 ] && shift
  mode=${args[0]}
  case $mode in
    check) run_check ;;
    ab) run_ab "${args[@]:1}" ;;
    run) run_one "${args[@]:1}" ;;
    prof) run_prof "${args[@]:1}" ;;
    pmc) run_pmc "${args[@]:1}" ;;
    *) echo "unknown mode $mode"; exit 2 ;;
  esac
  STEP=$((STEP + 1))
done
