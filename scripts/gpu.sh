#!/bin/bash
# The GPU jobs of this repo, by name (run on the box: gpurun -- 'bash scripts/gpu.sh JOB [ARGS]').
# Every GPU step runs under its own time limit and the first failure ends the job.
#
#   suite                 full GPU test suite + smoke() + the driver's bench line
#   tests  PYTEST_ARGS    selected GPU tests (e.g. tests/test_loopback.py)
#   bench  [N] [ARGS]     N runs of `bench.py --steps 200 --warmup 10 --no-extras ARGS`, ms per run
#   line   [ARGS]         one full driver bench line (extras included) -> gpurun_out/<tag>/bench.json
#   prof   MODEL [ARGS]   rocprofv3 kernel trace + per-dispatch breakdown of MODEL's step
#   pmc    COUNTERS CMD   one rocprofv3 --pmc pass (<= the per-block counter limits) over CMD
#   ab     VAR A B [ARGS] alternating bench runs under two values of an environment variable
#   sweep  VAR "V1 V2 .." [ARGS]  bench runs under each value in turn, ROUNDS passes
#   trees  ALT [ARGS]     alternating bench runs of another built source tree ALT against this one
#   tables "T1 T2[@VAR=V]" [ARGS]  alternating bench runs under GEMM tuning tables (DLS_GEMM_TUNING)
#   retune MODEL          exhaustive in-DAG GEMM refinement (benchmarks/refine_dag.py), then an A/B
#                         of the original table against the refined one
#   stamps                in-kernel phase stamps of the GPT-2 GEMM shapes (gpubin/gemm_stamps,
#                         built from benchmarks/gemm_stamps.hip)
# Output lands in gpurun_out/${TAG:-job}/.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
O="gpurun_out/${TAG:-job}"
mkdir -p "$O"
export DLS_SKIP_BUILD=1
job="$1"; shift

ms() { python -c "import json,sys;print(json.load(open(sys.argv[1]))['ms_per_step'])" "$1"; }

case "$job" in
  suite)
    timeout -k 10 1200 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
    tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
    tail -1 $O/smoke.log
    timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
    cut -c1-600 $O/bench.json
    ;;
  tests)
    timeout -k 10 1100 python -u -m pytest -x -v --timeout 240 --timeout-method thread "$@" > $O/pytest.log 2>&1; rc=$?
    grep -E "PASS|FAIL|ERROR|SKIP" $O/pytest.log | tail -60; tail -3 $O/pytest.log; exit $rc
    ;;
  bench)
    n="${1:-3}"; shift
    for i in $(seq "$n"); do
      timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-extras "$@" > $O/b$i.json 2> $O/b$i.err || { tail -20 $O/b$i.err; exit 4; }
      echo "run $i: $(ms $O/b$i.json) ms"
    done
    ;;
  line)
    timeout -k 10 600 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
    cut -c1-3000 $O/bench.json
    ;;
  prof)
    m="$1"; shift
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof_$m" -o k -- \
      python3 "$ROOT/bench.py" --model "$m" --steps 10 --warmup 3 --no-extras "$@" > "$ROOT/$O/prof_$m.log" 2>&1 \
      || { tail -20 "$ROOT/$O/prof_$m.log"; exit 7; }
    python3 "$ROOT/tools/analyze_trace.py" "$ROOT/$O/prof_$m/k_kernel_trace.csv" --steps 5 --per-dispatch > "$ROOT/$O/breakdown_$m.txt" 2>&1
    head -60 "$ROOT/$O/breakdown_$m.txt"
    ;;
  pmc)
    ctr="$1"; shift
    cd /tmp && export TMPDIR=/tmp
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$ROOT/$O/pmc" -o p -- "$@" > "$ROOT/$O/pmc.log" 2>&1 \
      || { tail -20 "$ROOT/$O/pmc.log"; exit 8; }
    ls "$ROOT/$O/pmc"
    ;;
  ab)
    var="$1"; a="$2"; b="$3"; shift 3
    for i in $(seq ${ROUNDS:-3}); do
      for v in "$a" "$b"; do
        env "$var=$v" timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-extras "$@" > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 3; }
        echo "$var=$v $(ms $O/ab.json)"
      done
    done
    ;;
  sweep)
    var="$1"; vals="$2"; shift 2
    for i in $(seq ${ROUNDS:-2}); do
      for v in $vals; do
        env "$var=$v" timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-extras "$@" > $O/sw.json 2> $O/sw.err || { tail -5 $O/sw.err; exit 3; }
        echo "$var=$v $(ms $O/sw.json)" | tee -a $O/sweep.txt > /dev/null
        echo "$var=$v $(ms $O/sw.json)"
      done
    done
    ;;
  trees)
    alt="$1"; shift
    for i in $(seq ${ROUNDS:-3}); do
      for t in "$alt" .; do
        timeout -k 10 300 python "$t/bench.py" --steps 200 --warmup 10 --no-extras "$@" > $O/t.json 2> $O/t.err || { tail -5 $O/t.err; exit 3; }
        echo "$t $(ms $O/t.json)"
      done
    done
    ;;
  tables)
    tabs="$1"; shift
    for i in $(seq ${ROUNDS:-3}); do
      for e in $tabs; do
        t=${e%%@*}; ev=""; [ "$e" != "$t" ] && ev=${e#*@}; ev=${ev//,/ }
        env DLS_GEMM_TUNING="$t" $ev timeout -k 10 300 python bench.py --no-extras --steps ${STEPS:-200} --warmup 10 "$@" \
          > $O/t.json 2> $O/t.err || { tail -5 $O/t.err; exit 3; }
        echo "$(basename $t) $ev $(ms $O/t.json)" | tee -a $O/tables.txt
      done
    done
    ;;
  retune)
    m="${1:-gpt2}"
    cp distributed_llm_scheduler_amd/ops/gemm_tuning.json $O/orig.json
    cp distributed_llm_scheduler_amd/ops/gemm_tuning.json $O/refined.json
    DLS_GEMM_TUNING=$O/refined.json timeout -k 10 900 python benchmarks/refine_dag.py --model $m --reps ${REPS:-20} \
      > $O/refine.json 2> $O/refine.err || { tail -20 $O/refine.err; exit 4; }
    for i in 1 2; do
      for t in refined orig; do
        DLS_GEMM_TUNING=$O/$t.json timeout -k 10 300 python bench.py --model $m --steps 100 --warmup 5 --no-extras \
          > $O/b_$t.json 2>/dev/null || exit 5
        echo "$t $(ms $O/b_$t.json)"
      done
    done
    ;;
  stamps)
    : > $O/stamps.txt
    for shape in "24 512 2304 768" "27 512 768 768" "27 512 768 3072" "17 512 3072 768" "24 512 768 3072" "34 512 50304 768"; do
      timeout -k 5 30 gpubin/gemm_stamps $shape >> $O/stamps.txt 2>&1 || { echo "FAILED $shape"; exit 3; }
    done
    cat $O/stamps.txt
    ;;
  *)
    echo "unknown job $job"; exit 2
    ;;
esac
