#!/bin/bash
# One parameterised GPU-box pass (replaces the per-round one-off scripts).
# Usage: bash tools/gpu_run.sh OUT STEP [STEP ...]
#   tests[:EXPR]   pytest -m gpu (optionally -k EXPR), stops the pass on failure
#   smoke          __graft_entry__.smoke()
#   bench[:ARGS]   python bench.py ARGS (comma-separated, e.g. bench:--steps,3,--no-latency)
#   voc:CFG        python bench.py --config CFG
#   prof[:ARGS]    rocprofv3 --kernel-trace --stats over bench.py ARGS
# Every GPU step has its own time limit; the first failure ends the pass.
set -e
OUT=${1:?OUT}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
for step in "$@"; do
  kind=${step%%:*}; arg=""; [ "$kind" != "$step" ] && arg=${step#*:}
  case $kind in
    tests)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread "${k[@]}" \
        > "$OUT/pytest_gpu.log" 2>&1 || { tail -80 "$OUT/pytest_gpu.log"; exit 1; }
      tail -3 "$OUT/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      tail -1 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 600 python bench.py ${arg//,/ } > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    voc)
      timeout -k 10 400 python bench.py --config "$arg" > "$OUT/$arg.json" 2> "$OUT/$arg.err" || { tail -30 "$OUT/$arg.err"; exit 1; }
      cat "$OUT/$arg.json" ;;
    prof)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$OUT/prof" -o run --output-format csv \
        -- python3 "$R/bench.py" ${arg//,/ } > "$R/$OUT/bench_prof.json" 2> "$R/$OUT/prof.err") || { tail -30 "$OUT/prof.err"; exit 1; }
      ls "$OUT/prof" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
