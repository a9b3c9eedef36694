set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_team.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_team2.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_team2.log; [ $rc -eq 0 ] || exit $rc
bash tools/team_stamps.sh || exit 1
SKIP_TESTS=1 WLS="ppo_defaults cfg1" STEPS=200 bash tools/team_round.sh
