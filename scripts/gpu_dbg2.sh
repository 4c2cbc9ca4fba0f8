cd $GRAFT_REPO_ROOT
B=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
for v in 1 2; do
MAGENT_LIB=$B/libmagent_par$v.so timeout -k 10 120 python scripts/debug_rollout.py 1 > gpurun_out/dbg$v.txt 2>&1 || exit 1
done
