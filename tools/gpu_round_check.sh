set -o pipefail
bash tools/gpu_check.sh || exit $?
bash tools/gpu_proxy_bench.sh px3 || exit $?
NRS="4 8" ALGOS=direct SLICES="32768 131072" timeout -k 10 300 bash tools/slice_sweep.sh
