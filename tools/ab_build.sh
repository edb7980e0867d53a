#!/bin/bash
# Builds libmsv_hip.so from a given git revision's csrc/ (or the working tree: rev ".") into
# ab/<name>/ (for tools/jobs/ab.sh); EXPERIMENTS=1 also instantiates the round-1 timing experiments
# (revisions up to a91649a only); PATCHES="tools/ab_patches/x.patch ..." applies A/B-only source changes (the
# experiment switches kept out of the product kernels since round 6, e.g. r05_msv_identity_e.patch, then
# EXTRA_DEVFLAGS=-DMSV_IDENTITY_E) to the copy before building:
#   [EXPERIMENTS=1] [PATCHES=...] [EXTRA_DEVFLAGS=...] bash tools/ab_build.sh <rev|.> <name>
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2
TMP=$(mktemp -d)
if [ "$REV" = "." ]; then
  mkdir -p "$TMP/hmm_fasta_viterbi_amd"
  cp -r "$ROOT/hmm_fasta_viterbi_amd/csrc" "$TMP/hmm_fasta_viterbi_amd/"
  cp -r "$ROOT/include" "$TMP/"
else
  git -C "$ROOT" archive "$REV" hmm_fasta_viterbi_amd/csrc include | tar -x -C "$TMP"
fi
for p in ${PATCHES:-}; do patch -s -d "$TMP" -p1 < "$ROOT/$p"; done
make -s -j8 EXPERIMENTS=${EXPERIMENTS:-0} -C "$TMP/hmm_fasta_viterbi_amd/csrc" "$TMP/hmm_fasta_viterbi_amd/lib/libmsv_hip.so" >/dev/null
mkdir -p "$ROOT/ab/$NAME"
cp "$TMP/hmm_fasta_viterbi_amd/lib/libmsv_hip.so" "$ROOT/ab/$NAME/"
rm -rf "$TMP"
echo "ab/$NAME/libmsv_hip.so from $REV"
