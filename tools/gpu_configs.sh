# The other single-GPU configs: bench lines and kernel traces for 64k and zipf.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg
for c in 64k zipf; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-e2e --no-file-crc --no-seek --no-snappy --no-lz4 --no-encode > gpurun_out/cfg/bench_$c.json 2> gpurun_out/cfg/bench_$c.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/cfg/trace_$c -o run -- python3 bench.py --config $c --steps 40 --warmup 3 --no-cpu-baseline --no-e2e --no-validate --no-file-crc --no-seek --no-snappy --no-lz4 --no-encode > gpurun_out/cfg/trace_bench_$c.json 2> gpurun_out/cfg/trace_$c.log
done
