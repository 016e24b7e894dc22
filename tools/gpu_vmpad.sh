#!/bin/bash
# A/B: K zero-length stores after the prefetch (vmcnt(K) at the staging wait) vs shipped.
CONFIGS="4k zipf" VARIANTS="full vmpad8 vmpad14" exec bash tools/gpu_r4l.sh
