# end-to-end self-play training rounds with the PyTorch algo drop-in on the batched engine
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/python
for E in 64 256; do
  timeout -k 10 600 python -m mfrl_amd.train_battle --algo mfq --n_round 2 --map_size 40 --max_steps 100 --envs $E --base_dir gpurun_out/train_E$E > gpurun_out/train_E$E.log 2>&1 || exit 1
done
