# GPU box: the whole -m gpu suite, then the 64k and 4k timings (kernel trace of the 64k bench)
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
timeout -k 10 300 python -u tools/abl_multi.py --rounds 3 --config 64k --blocks 65536 full > gpurun_out/t64k.log 2>&1
timeout -k 10 300 python -u tools/abl_multi.py --rounds 3 --config 4k full > gpurun_out/t4k.log 2>&1
timeout -k 10 300 python -u tools/abl_multi.py --rounds 3 --config 64k --blocks 65536 full bwnocrc bwnocopy > gpurun_out/t64k_abl.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
