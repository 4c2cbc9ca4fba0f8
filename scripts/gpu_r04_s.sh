# Round 4: k_rollout's launch timeline at 8192 envs for 2 and 4 steps per launch (the engine's choice is 2).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04s}
mkdir -p $O
export TMPDIR=/tmp
for S in 2 4; do
  MAGENT_LIB=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 200 \
      python scripts/timeline_rollout.py --envs 8192 --substeps $S --launches 3 > $O/tl_s$S.txt 2>&1 || { tail -20 $O/tl_s$S.txt; exit 1; }
  cat $O/tl_s$S.txt | grep -v amdgpu.ids
done
