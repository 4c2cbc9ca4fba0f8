# Round 5: the few-env stepper's snapshot split (MFX_STAMPS build, slots 24-27 from the first copying lane).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05ac}
mkdir -p $O
MAGENT_LIB=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 300 python scripts/stamps_few.py --envs 8 --sub 20 --launches 20 --snap > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
cat $O/stamps.txt
