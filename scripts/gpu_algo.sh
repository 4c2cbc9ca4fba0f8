set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/train
export PYTHONPATH=$GRAFT_REPO_ROOT/mean-field-multi-agent-reinforcement-learning_amd/python
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_algo_gpu.py > gpurun_out/algo_tests.log 2>&1 || { tail -40 gpurun_out/algo_tests.log; exit 1; }
timeout -k 10 500 python -u -m mfrl_amd.train_battle --algo mfq --n_round 2 --max_steps 400 --map_size 40 --envs 256 --base_dir gpurun_out/train/mfq40_e256 > gpurun_out/train/mfq40_e256.log 2>&1 || { tail -30 gpurun_out/train/mfq40_e256.log; exit 1; }
