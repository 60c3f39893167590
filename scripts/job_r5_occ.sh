set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_occ; mkdir -p $O
# the Mixtral-8x7B expert launches (8 experts x 128 routed rows; gate/up with SwiGLU, down): every config
timeout -k 10 600 python -u benchmarks/bench_grouped.py 128,28672,4096,s 128,4096,14336 > $O/grouped.jsonl 2>&1 || { tail $O/grouped.jsonl; exit 3; }
cat $O/grouped.jsonl
