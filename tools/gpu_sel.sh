# selected GPU tests: SEL = pytest args (files / -k), output gpurun_out/sel.log
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${SEL:-tests -m gpu} -q -x --timeout 240 --timeout-method thread > gpurun_out/sel.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/sel.log
exit $rc
