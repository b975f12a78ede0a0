#!/usr/bin/env bash
# One parameterized GPU-box runner (run through gpurun from the repo root):
#   gpurun --timeout 900 -- 'bash tools/gpu.sh <tag> <step> [<step> ...]'
# Steps (each under its own time limit; the first failure ends the call):
#   tests          pytest -m gpu (one process, per-test timeout)
#   pytest:ARGS    pytest ARGS -m gpu (e.g. pytest:tests/test_scan_prune.py)
#   pytestok:ARGS  the same, but failing tests do not end the call (pytest rc 1 only)
#   smoke          __graft_entry__.smoke()
#   bench[:ARGS]   python bench.py ARGS (default: --steps 5 --warmup 2); ARGS use ',' for spaces
#   stats[:ARGS]   rocprofv3 --kernel-trace --stats over bench.py ARGS
#   pmc:NAME:C1,C2,...[:ARGS]   one rocprofv3 --pmc pass (kernel trace only) over bench.py ARGS
#   py:SCRIPT,ARGS python SCRIPT ARGS (output to py<n>.json / py<n>.err)
#   env:K=V        export K=V for the following steps (e.g. env:K10S_LIB=build/libk10s_prof.so)

# Outputs go to gpurun_out/<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
DEF_BENCH="--steps,5,--warmup,2"

args_of() { echo "${1:-$DEF_BENCH}" | tr ',' ' '; }

for step in "$@"; do
  kind=${step%%:*}
  rest=""; [[ "$step" == *:* ]] && rest=${step#*:}
  echo "[gpu.sh] step $step"
  case $kind in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
        > "$O/pytest_gpu.log" 2>&1 || { echo "TESTS FAILED rc=$?"; tail -30 "$O/pytest_gpu.log"; exit 1; }
      tail -1 "$O/pytest_gpu.log" ;;
    pytest)
      n=$(ls "$O"/pytest_sel*.log 2>/dev/null | wc -l)
      timeout -k 10 600 python -u -m pytest $(args_of "$rest") -m gpu -x -v --timeout 180 --timeout-method thread \
        > "$O/pytest_sel$n.log" 2>&1 || { echo "PYTEST FAILED"; tail -30 "$O/pytest_sel$n.log"; exit 1; }
      tail -1 "$O/pytest_sel$n.log" ;;
    pytestok)   # like pytest, but a test failure is recorded and the next step still runs (a run that
                # times out or crashes still ends the call)
      n=$(ls "$O"/pytest_sel*.log 2>/dev/null | wc -l)
      timeout -k 10 600 python -u -m pytest $(args_of "$rest") -m gpu -v --timeout 180 --timeout-method thread \
        > "$O/pytest_sel$n.log" 2>&1; rc=$?
      tail -1 "$O/pytest_sel$n.log"
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "PYTEST rc=$rc: stop"; exit 1; fi ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { echo "SMOKE FAILED"; tail -20 "$O/smoke.log"; exit 1; }
      tail -4 "$O/smoke.log" ;;
    bench)
      n=$(ls "$O"/bench*.json 2>/dev/null | wc -l)
      timeout -k 10 900 python -u bench.py $(args_of "$rest") > "$O/bench$n.json" 2> "$O/bench$n.err" \
        || { echo "BENCH FAILED"; tail -20 "$O/bench$n.err"; exit 1; }
      tail -c 600 "$O/bench$n.json"; echo ;;
    stats)
      n=$(ls -d "$O"/stats*/ 2>/dev/null | wc -l); sd=stats; [ "$n" -gt 0 ] && sd=stats$n
      (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$sd" -o run \
        -- python3 "$R/bench.py" $(args_of "$rest") > "$O/$sd.json" 2> "$O/$sd.err") \
        || { echo "STATS FAILED"; tail -20 "$O/$sd.err"; exit 1; }
      find "$O/$sd" -name "*kernel_stats.csv" -exec cat {} \; ;;
    pmc)
      name=${rest%%:*}; r2=${rest#*:}; ctrs=${r2%%:*}; bargs=""; [[ "$r2" == *:* ]] && bargs=${r2#*:}
      (cd /tmp && timeout -k 10 -s KILL 600 rocprofv3 --kernel-trace --output-format csv -d "$O/pmc_$name" -o run \
        --pmc $(echo "$ctrs" | tr ',' ' ') -- python3 "$R/bench.py" $(args_of "$bargs") \
        > "$O/pmc_$name.json" 2> "$O/pmc_$name.err") || { echo "PMC $name FAILED"; tail -20 "$O/pmc_$name.err"; exit 1; }
      echo "PMC $name ok" ;;
    py)
      n=$(ls "$O"/py*.json 2>/dev/null | wc -l)
      timeout -k 10 600 python -u $(args_of "$rest") > "$O/py$n.json" 2> "$O/py$n.err" \
        || { echo "PY FAILED"; tail -20 "$O/py$n.err"; exit 1; }
      tail -c 1500 "$O/py$n.json"; echo ;;
    env)
      export "$rest"; echo "exported $rest" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu.sh] done"
