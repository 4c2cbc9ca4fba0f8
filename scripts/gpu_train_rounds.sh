# Self-play training rounds with the PyTorch algo drop-in: the BASELINE training configs
#   configs[1]: 40x40 Battle, MF-Q, one env (reference senario_battle.play loop through the drop-in magent)
#   configs[2]: 64x64 Battle, MF-AC, one env, then 64 envs on the batched engine
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/train
export PYTHONPATH=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/python
run() { name=$1; shift; timeout -k 10 900 python -m mfrl_amd.train_battle "$@" --base_dir gpurun_out/train/$name > gpurun_out/train/$name.log 2>&1 || { tail -20 gpurun_out/train/$name.log; exit 1; }; }
run mfq40_e1 --algo mfq --n_round 3 --map_size 40 --max_steps 400 --envs 1
run mfac64_e1 --algo mfac --n_round 2 --map_size 64 --max_steps 400 --envs 1
run mfac64_e64 --algo mfac --n_round 2 --map_size 64 --max_steps 400 --envs 64
run mfq40_e256 --algo mfq --n_round 2 --map_size 40 --max_steps 400 --envs 256
grep -h "TIME\|round" gpurun_out/train/*.log | tail -40
