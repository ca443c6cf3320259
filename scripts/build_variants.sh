#!/bin/bash
# A/B builds of the search kernels: scripts/build_variants.sh NAME "-DKNOB=.." [NAME "-D.."]...
# -> build/var/NAME/libbibfs.so (run a tool with LD_LIBRARY_PATH=build/var/NAME).
# VAR_SRC=<stem> varies csrc/hip/<stem>.hip instead of engine_kernels (e.g. tiny_engine).
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
cd "$ROOT"
make -s -j8 gpu >/dev/null
OBJS=$(ls build/obj/{io,gen,csr,cpu}/*.o | grep -v mpi_) 
SRC=${VAR_SRC:-engine_kernels}
OTHER=$(ls build/obj/hip/*.o build/obj/dist/*.o | grep -v "/$SRC.o")
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p build/var/$name
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -mcode-object-version=5 -munsafe-fp-atomics \
    -mllvm -amdgpu-atomic-optimizer-strategy=None -Icsrc/include -Icsrc/hip $flags -c csrc/hip/$SRC.hip -o build/var/$name/$SRC.o &
done
wait
for d in build/var/*/; do
  [ -f $d/$SRC.o ] || continue
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libbibfs.so $OBJS $OTHER $d/$SRC.o \
    -L/opt/rocm/lib -lamdhip64 -lhsa-runtime64 -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -lrccl -pthread
done
ls build/var
