# Same-box PMC of the round-1 library against the current one at one step per launch (and 4)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02/pmcr1
mkdir -p $O
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/build
for v in r1 cur; do
  lib=$L/libmagent_$v.so; [ $v = cur ] && lib=$L/libmagent.so
  MAGENT_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w_$v -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --substeps 1 --no-cpu-baseline > $O/w_$v.json 2> $O/w_$v.err || exit 1
  MAGENT_LIB=$lib timeout -k 10 200 python3 bench.py --steps 60 --substeps 1 --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.err || exit 1
done
timeout -k 10 200 python3 bench.py --steps 60 --substeps 4 --no-cpu-baseline > $O/b_cur4.json 2> $O/b_cur4.err || exit 1
