# round 6: tgemm main-loop schedule A/B (lab builds of the production kernel: s0 = compiler order,
# s1 = one fragment read per MFMA gap via sched_group_barrier, s2 = iglp_opt(0)) at the flagship's
# decode M, production plans only, PLAIN epilogue, rotated cold weights
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6l
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 0 1 2; do
  timeout -k 10 240 scripts/exp/bin/gemmlab_s$v 480 0 zzz > gpurun_out/r6l/s$v.jsonl 2>&1 || { tail -5 gpurun_out/r6l/s$v.jsonl; exit 1; }
  wc -l gpurun_out/r6l/s$v.jsonl
done
timeout -k 10 120 scripts/exp/bin/player 20 > gpurun_out/r6l/player.jsonl 2>&1 || { cat gpurun_out/r6l/player.jsonl; exit 1; }
cat gpurun_out/r6l/player.jsonl
