#!/bin/bash
# One parametrised GPU run (replaces the per-round gpu_r0*.sh one-offs). Steps run in the
# order given, each under its own time limit; the first failing GPU step ends the call.
#   TAG=r04a bash scripts/gpu_run.sh tests[:<pytest args>] smoke phases bench[:<bench args>]
#                                    profile[:<bench args>] rehearsal fe_prof cmd:<command>
# tests        python -m pytest tests -m gpu (or the given files / -k) -> <tag>_tests.log
# smoke        __graft_entry__.smoke()                                   -> <tag>_smoke.log
# phases       scripts/dstep_phases.py (debug build, k_dir_step stamps)  -> <tag>_phases.log
# bench        python bench.py [args]                                    -> <tag>_bench.log
# profile      scripts/profile.sh <tag> [args] (trace + PMC passes)      -> prof_<tag>/
# wcal         WRITE_SIZE calibration on known write streams   -> <tag>_wcal_*, wcal_<tag>/
# rehearsal    the 8-rank C4 group rehearsal under rocprof + per-rank kernel times
# fe_prof[:k,m] rocprof kernel stats of a general-degree solve at C3 (default (2, 0))
# ledger       k_dir_step store ledger (debug build, WRITE_SIZE per class) -> <tag>_ledger.json
# cmd:<c>      any command (e.g. cmd:"python scripts/direct_timing.py 18")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
mkdir -p gpurun_out
T=${TAG:-run}
step() {  # name timeout logfile command...
  local name=$1 t=$2 log=$3; shift 3
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 4 "$log"
  return $rc
}
for s in "$@"; do
  name=${s%%:*}; arg=""; [ "$name" != "$s" ] && arg=${s#*:}
  case $name in
    tests)
      # shellcheck disable=SC2086
      step tests 900 "gpurun_out/${T}_tests.log" python -u -m pytest ${arg:-tests} -m gpu -x -v \
        --timeout 120 --timeout-method thread || exit $? ;;
    smoke)
      step smoke 120 "gpurun_out/${T}_smoke.log" python -c 'import __graft_entry__ as g; g.smoke()' || exit $? ;;
    phases)
      step phases 120 "gpurun_out/${T}_phases.log" python scripts/dstep_phases.py || exit $? ;;
    bench)
      # shellcheck disable=SC2086
      step bench 300 "gpurun_out/${T}_bench.log" python bench.py $arg || exit $? ;;
    profile)
      # shellcheck disable=SC2086
      step profile 900 "gpurun_out/${T}_profile.log" bash scripts/profile.sh "$T" $arg || exit $? ;;
    rehearsal)
      TAG=$T step rehearsal 600 "gpurun_out/${T}_rehearsal.log" bash scripts/rehearsal_profile.sh || exit $?
      python scripts/rank_times.py "gpurun_out/prof_reh_$T/trace_kernel_trace.csv" 8 \
        > "gpurun_out/${T}_rank_times.txt" 2>&1; cat "gpurun_out/${T}_rank_times.txt" ;;
    fe_prof)
      mkdir -p "gpurun_out/prof_$T"
      (cd /tmp && export TMPDIR=/tmp && step fe_prof 300 "$R/gpurun_out/prof_$T/run.log" \
        rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$T" -o trace --output-format csv \
        -- python3 "$R/scripts/fe_timing.py" 15 15 "${arg:-2,0}") || exit $? ;;
    wcal)  # WRITE_SIZE against known write streams (scripts/micro/write_ceiling.hip)
      hipcc --offload-arch=gfx950 -O3 -o gpurun_out/write_ceiling scripts/micro/write_ceiling.hip || exit 1
      step wcal_time 120 "gpurun_out/${T}_wcal_time.log" gpurun_out/write_ceiling || exit $?
      (cd /tmp && export TMPDIR=/tmp && step wcal_pmc 120 "$R/gpurun_out/${T}_wcal_pmc.log" \
        rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/wcal_$T" -o pmc --output-format csv \
        -- "$R/gpurun_out/write_ceiling") || exit $? ;;
    ledger)  # k_dir_step's store ledger: one WRITE_SIZE pass per dropped store class
      for m in 0 1 2 4 16; do
        mkdir -p "gpurun_out/ledger_$T/m$m"
        (cd /tmp && export TMPDIR=/tmp NXHIP_LIB="$R/networks_fenicsx_amd/libnxhip_phase.so" \
          NXHIP_LEDGER=$m && step "ledger_m$m" 120 "$R/gpurun_out/ledger_$T/m$m/run.log" \
          rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/ledger_$T/m$m" -o pmc --output-format csv \
          -- python3 "$R/scripts/store_ledger.py" run 6) || exit $?
        f=$(find "gpurun_out/ledger_$T/m$m" -name 'pmc_counter_collection.csv' | head -n 1)
        [ -n "$f" ] && cp "$f" "gpurun_out/ledger_$T/m$m/pmc_counter_collection.csv" 2>/dev/null
      done
      python scripts/store_ledger.py summarize "gpurun_out/ledger_$T" > "gpurun_out/${T}_ledger.json" 2>&1
      cat "gpurun_out/${T}_ledger.json" ;;
    cmd)
      step cmd 600 "gpurun_out/${T}_cmd.log" bash -c "$arg" || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
