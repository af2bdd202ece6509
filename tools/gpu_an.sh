cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/an && timeout -k 10 600 python -u -m pytest tests/test_actor_gpu.py tests/test_config3_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/an/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/an/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_learner_prof.sh lp2
