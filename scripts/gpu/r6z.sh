# round 6: kernel tables of Llama-3-8B and Mixtral-8x7B serving through the current engine
set -o pipefail
cd $GRAFT_REPO_ROOT
export DLLM_VERBOSE=1
MODEL=llama-3-8b CONVS=128 STEPS=2 PROFILE=1 LIMIT=500 bash scripts/gpu/model_bench.sh && \
MODEL=mixtral-8x7b CONVS=64 STEPS=2 PROFILE=1 LIMIT=600 bash scripts/gpu/model_bench.sh
