#!/bin/bash
# Build libmini_nccl.so variants with different compile-time kernel constants into
# tools/variants/<name>/libmini_nccl.so (perf_test picks one up through LD_LIBRARY_PATH: the apps
# link with RUNPATH).  Usage: tools/build_variants.sh name:"-DMACRO=V ..." ...
set -e
R=$(cd $(dirname $0)/.. && pwd)
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  out=$R/tools/variants/$name; mkdir -p $out/build
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -I$R/include \
    -I$R/mini-nccl_amd/csrc $defs -c $R/mini-nccl_amd/csrc/kernels.hip -o $out/build/kernels.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -o $out/libmini_nccl.so $out/build/kernels.o \
    $R/mini-nccl_amd/build/comm.o $R/mini-nccl_amd/build/peerbuf.o $R/mini-nccl_amd/build/ipcreg.o $R/mini-nccl_amd/build/bootstrap.o $R/mini-nccl_amd/build/config.o \
    $R/mini-nccl_amd/build/api.o -shared -Wl,-Bsymbolic -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -lamdhip64 \
    -lrocprofiler-sdk-roctx -lhsa-runtime64 -pthread -lrt
  echo "built $name ($defs)"
done
