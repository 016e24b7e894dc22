# GPU box: snappy parity tests, then the codec step timing (A/B in one process)
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/codec_probe.py --steps 20 full ${VARIANTS:-} > gpurun_out/codec_ab.log 2>&1
