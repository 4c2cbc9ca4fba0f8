#!/bin/bash
# Round 6: the new rules tests (three-level rule, crowded kill_supply) against the reference build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06r
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rules_gpu.py > gpurun_out/r06r/tests.log 2>&1; rc=$?; tail -15 gpurun_out/r06r/tests.log; exit $rc
