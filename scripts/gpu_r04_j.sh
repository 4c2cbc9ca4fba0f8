# Round 4: the pipelined stepper's phase stamps, every step of a launch, with the real-time clock.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r04j}
mkdir -p $O
export TMPDIR=/tmp
for e in 8 64; do
  MAGENT_LIB=$PWD/mean-field-multi-agent-reinforcement-learning_amd/build/libmagent_stamps.so timeout -k 10 200 \
      python scripts/stamps_few.py --envs $e > $O/stamps_few_$e.txt 2>&1 || { tail -20 $O/stamps_few_$e.txt; exit 1; }
  cat $O/stamps_few_$e.txt
done
