#!/bin/bash
# One parametrised GPU job (run through gpurun from the repo root):
#   gpurun --timeout 900 -- 'bash tools/gpu_run.sh TAG STEP [STEP ...]'
# STEP is one of
#   tests           pytest -m gpu (one process, per-test timeout)
#   pytest:PATHS    pytest on the given test files / node ids
#   smoke           __graft_entry__.smoke()
#   bench[:ARGS]    python bench.py ARGS (default --steps 5 --warmup 1), JSON line -> gpurun_out/TAG_bench.json
#   stats[:ARGS]    rocprofv3 --kernel-trace --stats over bench.py ARGS -> gpurun_out/TAG_stats/
#   pmc:CNTRS[:ARGS] one rocprofv3 --pmc pass (counters comma-separated) over bench.py ARGS
#   py:SCRIPT[:ARGS] python SCRIPT ARGS
# Steps run in order; the job stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
idx=0
for step in "$@"; do
  idx=$((idx+1))
  kind=${step%%:*}; rest=${step#*:}; [ "$rest" = "$step" ] && rest=""
  echo "== $tag $step $(date +%T)"
  case $kind in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
             > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
           tail -3 gpurun_out/${tag}_tests.log ;;
    pytest) timeout -k 10 900 python -u -m pytest ${rest} -x -v --timeout 300 --timeout-method thread \
             > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
           tail -3 gpurun_out/${tag}_pytest.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 \
             || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
           tail -2 gpurun_out/${tag}_smoke.log ;;
    bench) args=${rest:-"--steps 5 --warmup 1"}
           timeout -k 10 900 python bench.py $args --detail gpurun_out/${tag}_bench_detail.json > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
             || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
           cut -c1-600 gpurun_out/${tag}_bench.json ;;
    stats) args=${rest:-"--steps 5 --warmup 1 --no-cpu-baseline --inflight 1"}
           st=${tag}_s${idx}
           timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/${st}_stats -o run -- \
             python3 bench.py $args --detail gpurun_out/${st}_detail.json > gpurun_out/${st}_stats.log 2>&1 || { tail -20 gpurun_out/${st}_stats.log; exit 1; }
           # keep the summaries only (the full kernel trace exceeds what gpurun copies back)
           for f in $(find /tmp/${st}_stats -name "*stats.csv"); do cp $f gpurun_out/${st}_$(basename $f); done
           ls gpurun_out/ | grep "^${tag}_" ;;
    pmc)   cn=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args="--steps 1 --warmup 0 --no-cpu-baseline --no-roofline --inflight 1"
           timeout -s KILL 300 rocprofv3 --pmc ${cn//,/ } --kernel-trace --output-format csv -d /tmp/${tag}_pmc_${cn%%,*} -o run -- \
             python3 bench.py $args --detail "" > gpurun_out/${tag}_pmc_${cn%%,*}.log 2>&1 || { tail -20 gpurun_out/${tag}_pmc_${cn%%,*}.log; exit 1; }
           # per-kernel summary only (the per-dispatch CSV is large)
           python tools/pmc_summary.py /tmp/${tag}_pmc_${cn%%,*} gpurun_out/${tag}_pmc_${cn%%,*}.json | tail -4 ;;
    py)    script=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
           timeout -k 10 900 python -u $script $args > gpurun_out/${tag}_$(basename $script .py).log 2>&1 \
             || { tail -30 gpurun_out/${tag}_$(basename $script .py).log; exit 1; }
           tail -15 gpurun_out/${tag}_$(basename $script .py).log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
