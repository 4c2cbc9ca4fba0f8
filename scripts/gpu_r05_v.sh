# Round 5: k_rollout phase stamps at 8192 envs (MFX_STAMPS build, one step per launch): install / write-back share
# and the launch's tail (envs resident over the launch).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05v}
mkdir -p $O
for E in 8192 131072; do
MAGENT_LIB=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 300 python scripts/stamps_battle.py --envs $E --steps 4 > $O/stamps$E.txt 2>&1 || { tail -20 $O/stamps$E.txt; exit 1; }
echo "== $E"; cat $O/stamps$E.txt
done
