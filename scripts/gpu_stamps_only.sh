cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MAGENT_LIB=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 300 python scripts/stamps_battle.py --envs 16384 > gpurun_out/stamps.txt 2>&1
