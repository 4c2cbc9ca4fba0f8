# Round 5: phase stamps after the wave-team rework (fused set_action / clear_dead, DPP wave_sum, mask-based moves and
# attacks): the few-env stepper (8 envs, 20-step launches) and k_rollout at 8192 envs (one step per launch).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05am}
mkdir -p $O
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so
MAGENT_LIB=$L timeout -k 10 300 python scripts/stamps_few.py --envs 8 --sub 20 --launches 20 --snap > $O/stamps_few.txt 2>&1 || { tail -20 $O/stamps_few.txt; exit 1; }
grep -v amdgpu.ids $O/stamps_few.txt
MAGENT_LIB=$L timeout -k 10 300 python scripts/stamps_battle.py --envs 8192 --steps 4 > $O/stamps8192.txt 2>&1 || { tail -20 $O/stamps8192.txt; exit 1; }
grep -v amdgpu.ids $O/stamps8192.txt
