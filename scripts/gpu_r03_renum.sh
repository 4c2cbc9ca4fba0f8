# Round 3: slot renumbering at clear_dead on the large-env path (clear_dead_renumber).
# Parity (large-env / queue-kernel rollout tests incl. the per-call-on-renumbered-state test), then an
# interleaved 256x256 A/B (MFX_RENUMBER=0 / 1, same box) and FETCH_SIZE / WRITE_SIZE passes of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/renum}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rollout_gpu.py \
    -k "large_env or bigq or small_e" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for v in 0 1; do
    MFX_RENUMBER=$v timeout -k 10 300 python bench.py --map 256 --agents 4096 --no-cpu-baseline \
        > $O/ab_${v}_$r.json 2> $O/ab_${v}_$r.err || { tail -20 $O/ab_${v}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/ab_${v}_$r.json')); print('renumber=$v', '%.4e' % d['value'], 'frac %.4f' % d['roofline']['frac'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'], 'check', d['check']['ok'])"
  done
done
for v in 0 1; do
  MFX_RENUMBER=$v timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f$v -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 32 --warmup 16 --no-cpu-baseline --check-envs 0 > $O/f$v.json 2> $O/f$v.err || exit 1
  MFX_RENUMBER=$v timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w$v -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 32 --warmup 16 --no-cpu-baseline --check-envs 0 > $O/w$v.json 2> $O/w$v.err || exit 1
  python3 scripts/pmc_kernels.py $O/f$v/run_counter_collection.csv FETCH_SIZE 2 > $O/pmcf$v.json || exit 1
  python3 scripts/pmc_kernels.py $O/w$v/run_counter_collection.csv WRITE_SIZE 2 > $O/pmcw$v.json || exit 1
  python3 -c "import json; f=json.load(open('$O/pmcf$v.json'))['kernels']['k_rollout_bigq']['avg_kib_last']; w=json.load(open('$O/pmcw$v.json'))['kernels']['k_rollout_bigq']['avg_kib_last']; b=json.load(open('$O/f$v.json')); u=b['roofline']['units_per_launch']; print('renumber=$v fetch x2 %.3f GB write %.3f GB per launch, %.0f B per agent-step' % (2*f*1024/1e9, w*1024/1e9, (2*f+w)*1024/u))"
  rm -f $O/f$v/run_counter_collection.csv $O/w$v/run_counter_collection.csv
done
