#!/bin/bash
# Dump the gfx950 assembly of every MSV and Viterbi kernel translation unit into $1 (one .s per TU), for
# instruction-for-instruction comparisons of a source change (tools/isa_compare.py).
set -e
OUT=${1:?usage: tools/isa_dump.sh OUTDIR}
HERE=$(cd "$(dirname "$0")/../hmm_fasta_viterbi_amd/csrc" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
mkdir -p "$OUT"
FLAGS="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -fno-honor-nans -fno-slp-vectorize -ffp-contract=off -I$ROOT/include -I$HERE --cuda-device-only -S"
for k in 0 1 2 3 4 5 6 7; do
  /opt/rocm/bin/hipcc $FLAGS -DMSV_PART=$k -DMSV_PART_INC="\"msv_variants_$k.inc\"" "$HERE/msv_kernel_part.hip" -o "$OUT/part$k.s" &
done
/opt/rocm/bin/hipcc $FLAGS "$HERE/msv_kernel.hip" -o "$OUT/msv_kernel.s" &
/opt/rocm/bin/hipcc $FLAGS "$HERE/msv_coop.hip" -o "$OUT/msv_coop.s" &
/opt/rocm/bin/hipcc $FLAGS "$HERE/vit_kernel.hip" -o "$OUT/vit_kernel.s" &
/opt/rocm/bin/hipcc $FLAGS "$HERE/vit_team.hip" -o "$OUT/vit_team.s" &
wait
