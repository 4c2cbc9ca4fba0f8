# Round-2 health check of the committed tree: GPU tests, smoke, the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
