#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/gpu_profile.sh r02i
