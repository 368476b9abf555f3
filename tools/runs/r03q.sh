set -o pipefail
OUT=gpurun_out/r03q bash tools/dense_ab.sh
