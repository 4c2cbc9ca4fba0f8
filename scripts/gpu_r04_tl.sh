# Round 4: k_rollout launch timeline (stamp build) at 8192 / 32768 / 131072 envs, 20 steps per launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04tl}
mkdir -p $O
export TMPDIR=/tmp
L=mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so
for E in 8192 32768 131072; do
MAGENT_LIB=$L timeout -k 10 200 python scripts/timeline_rollout.py --envs $E --substeps 20 > $O/tl_$E.txt 2>&1 || { tail -20 $O/tl_$E.txt; exit 1; }
cat $O/tl_$E.txt
done
