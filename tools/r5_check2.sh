#!/bin/bash
# NT-store A/B (reversed order) then the GPU suite and smoke() on the shipped build
set -o pipefail
timeout -k 10 900 bash tools/r5_nt.sh || exit 1
bash tools/r5_check.sh
