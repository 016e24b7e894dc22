set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-file-crc --no-seek --no-snappy --no-lz4 > gpurun_out/bench_enc.json 2> gpurun_out/bench_enc.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_enc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-file-crc --no-seek --no-snappy --no-lz4 --no-validate > $GRAFT_REPO_ROOT/gpurun_out/bench_enc_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench_enc_prof.err
