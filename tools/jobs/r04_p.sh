# Round 4 job P: the MSV kernel's 64-lane shift as one wave_shr:1 DPP move (G = 64 batch plans and the
# cooperative single-sequence plan; the bench plans' ISA is unchanged): the whole GPU suite, then A/B against
# the previous build (ab/mbase) on small batches (64-lane plans) and the reference's benchmark programs.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --n 1000 --rounds 4 ab/mbase/libmsv_hip.so hmm_fasta_viterbi_amd/lib/libmsv_hip.so > $O/ab_1400_n1000.jsonl 2> $O/ab.err
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --profile 2405.hmm --n 600 --rounds 4 ab/mbase/libmsv_hip.so hmm_fasta_viterbi_amd/lib/libmsv_hip.so > $O/ab_2405_n600.jsonl 2>> $O/ab.err
for r in 1 2 3; do
  for lib in ab/mbase/libmsv_hip.so hmm_fasta_viterbi_amd/lib/libmsv_hip.so; do
    MSV_LIB_PATH=$lib timeout -k 10 200 python tools/bench_reference_programs.py | sed "s#^{#{\"lib\": \"$lib\", #" >> $O/ab_reference_programs.jsonl
  done
done
timeout -k 10 300 python tools/vit_tune.py --profile 2405.hmm --n 3000 --lmin 300 --lmax 500 --insert-mode 1 --rounds 2 --variants vit_s38_t0gi,vit_s38_t7gw4i,vit_s64_t0gi > $O/tune_isc_2405.jsonl 2> $O/tune.err
timeout -k 10 300 python tools/vit_tune.py --profile 2138.hmm --n 3000 --lmin 300 --lmax 500 --insert-mode 1 --rounds 2 --variants vit_s34_t7gw4i,vit_s38_t7gw4i,vit_s38_t0gi > $O/tune_isc_2138.jsonl 2>> $O/tune.err
timeout -k 10 300 python tools/vit_tune.py --profile 1705.hmm --n 3000 --lmin 300 --lmax 500 --insert-mode 1 --rounds 2 --variants vit_s28_t0gi,vit_s32_t0gi > $O/tune_isc_1705.jsonl 2>> $O/tune.err
