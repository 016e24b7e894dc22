# GPU box: snappy ring-kernel variants (A/B in one process), then the quick bench line
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/codec_probe.py --steps 20 full unified > gpurun_out/codec_ab.log 2>&1
