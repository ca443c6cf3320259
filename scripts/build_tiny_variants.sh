#!/bin/bash
# A/B builds of the small-graph server: scripts/build_tiny_variants.sh NAME "-DKNOB=.." [NAME "-D.."]...
# -> build/var/NAME/libbibfs.so (run with LD_LIBRARY_PATH=build/var/NAME).
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
cd "$ROOT"
make -s -j8 gpu >/dev/null
OBJS=$(ls build/obj/{io,gen,csr,cpu}/*.o | grep -v mpi_)
OTHER=$(ls build/obj/hip/*.o build/obj/dist/*.o | grep -v tiny_engine)
rm -rf build/var
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p build/var/$name
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -mcode-object-version=5 -munsafe-fp-atomics \
    -mllvm -amdgpu-atomic-optimizer-strategy=None -Icsrc/include -Icsrc/hip $flags -c csrc/hip/tiny_engine.hip -o build/var/$name/tiny_engine.o &
done
wait
for d in build/var/*/; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libbibfs.so $OBJS $OTHER $d/tiny_engine.o \
    -L/opt/rocm/lib -lamdhip64 -lhsa-runtime64 -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -lrccl -pthread
done
ls build/var
