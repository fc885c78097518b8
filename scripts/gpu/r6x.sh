# round 6: the other model families through the current engine (routed bench lines, no profile)
set -o pipefail
cd $GRAFT_REPO_ROOT
export DLLM_VERBOSE=1
MODEL=llama-3-8b CONVS=128 STEPS=2 PROFILE=0 LIMIT=500 bash scripts/gpu/model_bench.sh && \
MODEL=phi3-mini CONVS=128 STEPS=2 PROFILE=0 LIMIT=500 bash scripts/gpu/model_bench.sh && \
MODEL=mixtral-8x7b CONVS=64 STEPS=2 PROFILE=0 LIMIT=600 bash scripts/gpu/model_bench.sh
