#!/bin/bash
# INTEGRATION.md §2, literally: the swap a maintainer makes in the reference tree, applied to a scratch copy of
# /root/reference (never to /root/reference itself, never inside this repository), then the reference's own
# CMake build and ctest.  Deletes the reference's class sources, replaces algorithms/CMakeLists.txt and
# data_readers/CMakeLists.txt with INTERFACE targets on include/drop_in + include + libmsv_hip.so, and keeps every
# caller source and the top-level CMakeLists.txt (-Wall -Wextra -pedantic -Werror) as they are.
#
#   bash tests/ref_callers/cmake_swap.sh [WORKDIR]    -> builds WORKDIR/src/build; runs the parser tests (CPU)
#   GPU=1 bash tests/ref_callers/cmake_swap.sh ...     -> also runs test_MSV through ctest (needs an MI355X)
set -euo pipefail
REF=${REF:-/root/reference}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
WORK=${1:-$(mktemp -d)}
mkdir -p "$WORK"
SRC=$WORK/src
rm -rf "$SRC"
cp -r "$REF" "$SRC"

# 1. the reference's own MSV class and parsers leave the build (a quoted #include looks in the including file's
#    directory first, so a left-over MSV_HMM.hpp beside test_MSV.cpp would shadow the library's)
rm -f "$SRC"/algorithms/MSV_HMM.hpp "$SRC"/algorithms/MSV_HMM.cpp "$SRC"/algorithms/MSV_kernels.cl \
      "$SRC"/algorithms/MSV_spec_kernels.cl "$SRC"/data_readers/Profile_HMM.hpp "$SRC"/data_readers/Profile_HMM.cpp \
      "$SRC"/data_readers/FASTA_protein_sequences.hpp "$SRC"/data_readers/FASTA_protein_sequences.cpp

# 2. the two libraries become INTERFACE targets on this engine (the executables and tests are the reference's)
cat > "$SRC"/algorithms/CMakeLists.txt <<EOF
cmake_minimum_required(VERSION 3.15)
project(algorithms)

add_library(algorithms INTERFACE)
target_include_directories(algorithms INTERFACE $ROOT/include/drop_in $ROOT/include)
target_link_libraries(algorithms INTERFACE $ROOT/hmm_fasta_viterbi_amd/lib/libmsv_hip.so)

add_executable(test_MSV test_MSV.cpp)
target_link_libraries(test_MSV algorithms)
target_link_libraries(test_MSV data_readers)
target_link_libraries(test_MSV stdc++fs)

add_test(test_MSV test_MSV)

add_executable(benchmark_MSV benchmark_helper.hpp benchmark_MSV.cpp)
target_link_libraries(benchmark_MSV algorithms)
target_link_libraries(benchmark_MSV data_readers)
target_link_libraries(benchmark_MSV stdc++fs)

add_executable(benchmark_MSV_1400 benchmark_helper.hpp benchmark_MSV_1400.cpp)
target_link_libraries(benchmark_MSV_1400 algorithms)
target_link_libraries(benchmark_MSV_1400 data_readers)
EOF
cat > "$SRC"/data_readers/CMakeLists.txt <<EOF
cmake_minimum_required(VERSION 3.15)
project(data_readers)

add_library(data_readers INTERFACE)
target_include_directories(data_readers INTERFACE $ROOT/include/drop_in $ROOT/include)
target_link_libraries(data_readers INTERFACE $ROOT/hmm_fasta_viterbi_amd/lib/libmsv_hip.so)

add_executable(test_hmm_parsing test_hmm_parsing.cpp)
target_link_libraries(test_hmm_parsing data_readers)
target_link_libraries(test_hmm_parsing stdc++fs)

add_executable(test_fasta_parsing test_fasta_parsing.cpp)
target_link_libraries(test_fasta_parsing data_readers)
target_link_libraries(test_fasta_parsing stdc++fs)

add_test(test_hmm_parsing test_hmm_parsing)
add_test(test_fasta_parsing_test test_fasta_parsing)
EOF

# 3. the reference's build (compile_clang_in_build_dir.sh:1-15 with g++, Debug so the asserts are live; -march=native
#    from the top-level CMakeLists.txt stays) and its tests, run from the build directories as its scripts do
mkdir -p "$SRC"/build
cp -r "$SRC"/profile_HMMs "$SRC"/FASTA_files "$SRC"/build/
cmake -S "$SRC" -B "$SRC"/build -DCMAKE_BUILD_TYPE=Debug -DCMAKE_CXX_COMPILER=g++ > "$WORK"/cmake.log 2>&1
make -C "$SRC"/build -j4 > "$WORK"/make.log 2>&1
if [ "${GPU:-0}" = 1 ]; then
  ctest --test-dir "$SRC"/build --output-on-failure
else
  ctest --test-dir "$SRC"/build --output-on-failure -R parsing
fi
echo "cmake swap OK: $SRC/build"
