set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 -k "sample or engine or graph or prefix or tinyllama or argmax" > gpurun_out/pytest_sampler.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_sampler.log; [ $rc -eq 0 ] || exit $rc
STEPS=8 WARMUP=2 bash scripts/ab_args.sh "" 
DLLM_FUSED_SAMPLER=0 STEPS=8 WARMUP=2 bash scripts/ab_args.sh ""
