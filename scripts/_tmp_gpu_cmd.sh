STEPS=8 WARMUP=2 bash scripts/ab_args.sh "" "--groups 4" "--groups 8" "--groups 16" ""
