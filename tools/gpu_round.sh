# Round check on the GPU box: GPU tests, smoke, full bench line, kernel trace of the bench.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/gputest.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r2/bench.json 2> gpurun_out/r2/bench.err
