# Round check on the GPU box: GPU tests, smoke, full bench line, kernel traces of the bench
# (decode: 40 timed steps; side measurements: codecs, encode), all under gpurun_out/r2.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/r2/gputest.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r2/bench.json 2> gpurun_out/r2/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r2/trace -o run -- python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-e2e --no-validate --no-snappy --no-lz4 --no-file-crc --no-seek --no-encode > gpurun_out/r2/trace_bench.json 2> gpurun_out/r2/trace.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r2/trace_side -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-validate > gpurun_out/r2/trace_side.json 2> gpurun_out/r2/trace_side.log
