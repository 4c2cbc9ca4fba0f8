# 256x256 (configs[4]): XCD-aware observation item lists (MFX_ITEM_XCD=1, default) against one shared
# list (MFX_ITEM_XCD=0): parity tests, interleaved bench A/B, FETCH_SIZE / WRITE_SIZE per kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_rollout_gpu.py -k "large" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for x in 1 0; do
    MFX_ITEM_XCD=$x timeout -k 10 200 python bench.py --map 256 --agents 4096 --steps 40 --warmup 5 --no-cpu-baseline > $O/b_x${x}_$r.json 2> $O/b_x${x}_$r.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/b_x${x}_$r.json')); print('xcd=$x', '%.4g'%d['value'], '%.3f'%d['roofline']['frac'])"
  done
done
for x in 1 0; do
  MFX_ITEM_XCD=$x timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f$x -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 20 --warmup 4 --no-cpu-baseline > /dev/null 2> $O/f$x.err || exit 1
  python3 scripts/pmc_kernels.py $O/f$x/run_counter_collection.csv FETCH_SIZE 40 > $O/fetch_x$x.json || exit 1
  MFX_ITEM_XCD=$x timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w$x -o run --output-format csv -- python3 bench.py --map 256 --agents 4096 --steps 20 --warmup 4 --no-cpu-baseline > /dev/null 2> $O/w$x.err || exit 1
  python3 scripts/pmc_kernels.py $O/w$x/run_counter_collection.csv WRITE_SIZE 40 > $O/write_x$x.json || exit 1
  rm -f $O/f$x/run_counter_collection.csv $O/w$x/run_counter_collection.csv
done
cat $O/fetch_x1.json $O/fetch_x0.json
