set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_b; mkdir -p $O
# Llama-3-8B gate/up on the whole-round 256x224 tile (config 37) vs the table's choice, same box
ROUNDS=3 STEPS=30 TAG=r5_b bash scripts/gpu.sh tables "distributed_llm_scheduler_amd/ops/gemm_tuning.json benchmarks/tuning_ab/llama_gateup_cfg37.json" --model llama3-8b || exit 3
# BASELINE multi-GPU configs at full size through the single-GPU harness, device transport
timeout -k 10 900 python -u benchmarks/loopback_configs.py --configs gpt2m_cap_eft,gpt2m_cap,llama_pipeline,mixtral_expert --transport device --steps 5 > $O/configs_device.jsonl 2> $O/configs_device.err || { tail -20 $O/configs_device.err; exit 4; }
cut -c1-700 $O/configs_device.jsonl
