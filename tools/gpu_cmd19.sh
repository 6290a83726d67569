set -o pipefail
run() { echo "== n=$1 $2 $3"; timeout -k 10 200 python tools/debug_hang.py "$@" 2>&1 | grep -v "^\[Gloo\]" | tail -12; }
run 8 '[{"count":1048581,"algo":1},{"dtype":"bf16","count":524291,"inplace":true,"algo":1,"seed":9}]' '{"MINI_NCCL_CHANNELS":"16"}'
run 8 '[{"dtype":"bf16","count":524291,"inplace":true,"algo":1,"seed":9}]' '{"MINI_NCCL_CHANNELS":"16"}'
run 8 '[{"dtype":"bf16","count":524291,"inplace":false,"algo":1,"seed":9}]' '{"MINI_NCCL_CHANNELS":"16"}'
run 8 '[{"dtype":"f32","count":524291,"inplace":true,"algo":1,"seed":9}]' '{"MINI_NCCL_CHANNELS":"16"}'
run 4 '[{"dtype":"bf16","count":524291,"inplace":true,"algo":1,"seed":9}]' '{"MINI_NCCL_CHANNELS":"16"}'
exit 0
