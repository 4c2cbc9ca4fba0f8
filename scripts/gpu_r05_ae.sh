# Round 5: where the few-env policy phase's 3.9K-cycle prologue goes (MFX_STAMPS build, slots 9-11).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05ae}
mkdir -p $O
MAGENT_LIB=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 300 python scripts/stamps_few.py --envs 8 --sub 20 --launches 20 --snap > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
grep -E "split|<= 64" $O/stamps.txt
