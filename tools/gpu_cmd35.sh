set -o pipefail
make -C mini-nccl_amd > gpurun_out/build.log 2>&1 || exit 3
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined -Wno-unused-result -pthread -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -Imini-nccl_amd/csrc -o gpurun_out/abi_selftest tests/native/abi_selftest.cpp mini-nccl_amd/csrc/{api,comm,bootstrap,config}.cpp mini-nccl_amd/build/kernels.o -L/opt/rocm/lib -lamdhip64 -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib || exit 4
MINI_NCCL_PORT=29888 ASAN_OPTIONS=detect_leaks=0:use_sigaltstack=0 timeout -k 10 120 gpurun_out/abi_selftest > gpurun_out/abi.out 2> gpurun_out/abi.err; echo "rc=$?"
cat gpurun_out/abi.out; tail -40 gpurun_out/abi.err
rm -f gpurun_out/abi_selftest
