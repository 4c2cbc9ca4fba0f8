#!/bin/bash
# Round 6 final refresh after the hygiene rebuild: the whole GPU suite and smoke, then part 2 (traces + PMC passes,
# the build-keyed pmc files, the bench line with traffic).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r06_final_c}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --durations=15 --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
OUT=$O/b bash scripts/gpu_r06_final_b.sh
