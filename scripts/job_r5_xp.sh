set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_xp; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u benchmarks/loopback_configs.py --configs mixtral_expert --transport device --steps 3 > $O/run.jsonl 2> $O/run.err || { tail -20 $O/run.err; exit 4; }
cut -c1-600 $O/run.jsonl
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -c1-220
