set -e
D=gpurun_out/r6w; mkdir -p $D
timeout -k 10 200 python bench.py --steps 8 --warmup 2 > $D/headline.json
timeout -k 10 200 python bench.py --workload env --envs 64 --height 16 --width 20 --hist 32 --steps 200 --warmup 20 > $D/config1_env_64.json
timeout -k 10 200 python bench.py --envs 1024 --steps 10 --warmup 3 > $D/config2_1024x50.json
timeout -k 10 200 python bench.py --workload env --envs 4096 --height 84 --width 84 --hist 4 --steps 200 --warmup 5 > $D/config3_env_84x84_4096.json
timeout -k 10 300 python bench.py --envs 4096 --height 84 --width 84 --hist 4 --steps 2 --warmup 1 --no-cpu > $D/config3_acting_84x84_4096x50.json
timeout -k 10 200 python bench.py --envs 4096 --sims 200 --dyn-dtype fp16 --steps 3 --warmup 1 --no-cpu > $D/config5_4096x200_fp16dyn.json
timeout -k 10 200 python bench.py --envs 4096 --sims 200 --steps 3 --warmup 1 --no-cpu > $D/config5_4096x200_bf16.json
timeout -k 10 200 python bench.py --workload learner --dtype bf16 --steps 10 --warmup 3 > $D/learner_bf16.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_learner -o run -- python3 bench.py --workload learner --dtype bf16 --steps 6 --warmup 2 --no-cpu > $D/prof_learner.out 2>&1
MZBA_DIST_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 8 --envs 4096 --steps 3 --warmup 1 > $D/selflaunch_n8.json
