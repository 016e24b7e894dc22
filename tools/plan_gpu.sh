# Write-side plan A/B on the GPU box: parity tests on the shipped plan kernels and on the
# alternatives (TPZ_PLAN_BISECT: bisection only; TPZ_PLAN_GLOBAL_WALK: the global-memory chain walks),
# then rocprofv3 kernel traces of tools/plan_probe.py for each.
set -e
mkdir -p gpurun_out/plan
export TMPDIR=/tmp
T="python -u -m pytest tests/test_gpu_encode.py -x -q --timeout 170 --timeout-method thread"
timeout -k 10 300 $T > gpurun_out/plan/test_new.log 2>&1
TPZ_PLAN_BISECT=1 timeout -k 10 300 $T -k "random or chunk or long or config" > gpurun_out/plan/test_bisect.log 2>&1
TPZ_PLAN_GLOBAL_WALK=1 timeout -k 10 300 $T -k "random or chunk or long or config" > gpurun_out/plan/test_old.log 2>&1
P="rocprofv3 --kernel-trace --stats --output-format csv -o run"
timeout -k 10 200 $P -d gpurun_out/plan/new -- python3 tools/plan_probe.py > gpurun_out/plan/probe_new.log 2>&1
TPZ_PLAN_BISECT=1 timeout -k 10 200 $P -d gpurun_out/plan/bisect -- python3 tools/plan_probe.py > gpurun_out/plan/probe_bisect.log 2>&1
TPZ_PLAN_GLOBAL_WALK=1 timeout -k 10 200 $P -d gpurun_out/plan/old -- python3 tools/plan_probe.py > gpurun_out/plan/probe_old.log 2>&1
timeout -k 10 200 $P -d gpurun_out/plan/zipf -- python3 tools/plan_probe.py --config zipf > gpurun_out/plan/probe_zipf.log 2>&1
TPZ_PLAN_BISECT=1 timeout -k 10 200 $P -d gpurun_out/plan/zipf_bisect -- python3 tools/plan_probe.py --config zipf > gpurun_out/plan/probe_zipf_bisect.log 2>&1
timeout -k 10 200 $P -d gpurun_out/plan/64k -- python3 tools/plan_probe.py --config 64k --blocks 65536 > gpurun_out/plan/probe_64k.log 2>&1
