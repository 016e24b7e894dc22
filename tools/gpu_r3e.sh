set -o pipefail
TESTS=tests TEST_TIMEOUT=300 VARIANTS="full cticket cprev" CONFIGS="64k zipf" ROUNDS=5 bash tools/gpu_ab.sh && mkdir -p gpurun_out/r3e && timeout -k 10 300 python3 -u tools/enc_probe.py --steps 10 full ec2 ec8 full ec2 ec8 full ec2 ec8 > gpurun_out/r3e/enc_probe.jsonl 2> gpurun_out/r3e/enc_probe.err
