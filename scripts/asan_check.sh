#!/bin/bash
# Host-code sanitizer run (SURVEY.md §5 "race detection / sanitizers"):
# build core, CPU engines, MPI engines and CLI tools with
# -fsanitize=address,undefined (make asan -> build-asan/), then run the
# not-gpu tests that drive those binaries, plus direct CLI runs over the
# reference graph shapes, edge cases and the MPI engines at np = 1..4.
# Any sanitizer report fails the run (halt_on_error / -fno-sanitize-recover).
set -euo pipefail
cd "$(dirname "$0")/.."
make -j8 asan > /dev/null
export BIBFS_BIN_DIR=$PWD/build-asan/bin
# MPICH keeps allocations alive until exit: leak checking only for non-MPI tools
export ASAN_OPTIONS=halt_on_error=1:abort_on_error=0:detect_leaks=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
B=$BIBFS_BIN_DIR
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
$B/bibfs_gen --type gnp --n 100000 --seed 6 --out "$tmp/100k.bin" > /dev/null
$B/bibfs_gen --type rmat --n 65536 --m 1048576 --seed 3 --out "$tmp/rmat.bin" > /dev/null
for args in "$tmp/100k.bin 0 99999" "$tmp/100k.bin 7 7" "$tmp/rmat.bin 1 4242" "gnp:1000::1 0 999" \
            "gnp:200000::2 0 199999 --json" "kron:14:16:3 3 77 --direction bottomup"; do
  $B/bibfs_serial $args > /dev/null
done
( $B/bibfs_serial "$tmp/missing.bin" 0 1 > /dev/null 2>&1 && exit 1 ) || true   # error path, no report
export ASAN_OPTIONS=halt_on_error=1:detect_leaks=0
for np in 1 2 3 4; do
  /opt/conda/bin/mpiexec -n $np $B/second_try "$tmp/100k.bin" 0 99999 > /dev/null
  /opt/conda/bin/mpiexec -n $np $B/mpi_queue_bibfs "$tmp/100k.bin" 0 99999 > /dev/null
done
python -m pytest -q -m "not gpu" tests/test_cli_tools.py tests/test_mpi_cpu.py tests/test_io.py tests/test_scripts.py
echo "asan_check: clean"
