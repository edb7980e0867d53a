// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" driver around the reference's OWN CPU path, compiled from the reference
// sources where they lie (/root/reference/{algorithms,data_readers}) by oracle/Makefile into
// oracle/_ref/libref_msv.so.  Nothing from the reference is copied into this repository; this
// file only calls the reference classes:
//   Profile_HMM(path)                      data_readers/Profile_HMM.cpp:48-60
//   FASTA_protein_sequences(path)          data_readers/FASTA_protein_sequences.cpp:9-44
//   MSV_HMM(hmm).run_on_sequence(seq)      algorithms/MSV_HMM.cpp:35-57, 74-113
//
// Used for (1) generating the golden fixtures in tests/golden (oracle/make_golden.py) and
// (2) the "reference" CPU baseline leg of bench.py, timed on the GPU box's host cores with one
// MSV_HMM instance per std::thread (the reference instance is not thread-safe, MSV_HMM.hpp:33-34).
#include "FASTA_protein_sequences.hpp"
#include "MSV_HMM.hpp"
#include "Profile_HMM.hpp"

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace {
const char kLetters[] = "ACDEFGHIKLMNPQRSTVWY";
}

extern "C" {

// Scores every sequence of a FASTA file (after the reference's own filter) with run_on_sequence.
// Returns the number of sequences, writes min(n, cap) scores and lengths (excluding '#').
long ref_score_fasta(const char* hmm_path, const char* fasta_path, float* scores, uint64_t* lengths, long cap) {
    auto fasta = FASTA_protein_sequences(fasta_path);
    auto msv = MSV_HMM(Profile_HMM(hmm_path));
    long n = static_cast<long>(fasta.sequences.size());
    for (long i = 0; i < n && i < cap; ++i) {
        scores[i] = msv.run_on_sequence(fasta.sequences[i]);
        lengths[i] = fasta.sequences[i].size() - 1;
    }
    return n;
}

// Concatenated '#'-prefixed sequences of the reference FASTA parser, '\n'-separated.
// Returns the number of bytes needed (call with cap=0 first).
long ref_fasta_dump(const char* fasta_path, char* out, long cap) {
    auto fasta = FASTA_protein_sequences(fasta_path);
    std::string all;
    for (auto& s : fasta.sequences) {
        all += s;
        all += '\n';
    }
    if (out && cap >= static_cast<long>(all.size()) + 1) std::memcpy(out, all.c_str(), all.size() + 1);
    return static_cast<long>(all.size()) + 1;
}

// Parsed profile fields (Profile_HMM.hpp:21-49). match/insert: [model_length][20], trans: [model_length][7].
long ref_hmm_dump(const char* hmm_path, char* name, long name_cap, float* stats6, float* match, float* insert,
                  float* trans, long cap_nodes) {
    auto h = Profile_HMM(hmm_path);
    if (name && name_cap > 0) {
        std::strncpy(name, h.name.c_str(), name_cap - 1);
        name[name_cap - 1] = 0;
    }
    if (stats6) {
        stats6[0] = h.stats_local_msv_mu;
        stats6[1] = h.stats_local_msv_lambda;
        stats6[2] = h.stats_local_viterbi_mu;
        stats6[3] = h.stats_local_viterbi_lambda;
        stats6[4] = h.stats_local_forward_theta;
        stats6[5] = h.stats_local_forward_lambda;
    }
    long M = static_cast<long>(h.model_length);
    for (long i = 0; i < M && i < cap_nodes; ++i) {
        for (int j = 0; j < 20; ++j) {
            if (match) match[i * 20 + j] = h.match_emissions[i][j];
            if (insert) insert[i * 20 + j] = h.insert_emissions[i][j];
        }
        for (int j = 0; j < 7; ++j)
            if (trans) trans[i * 7 + j] = h.transitions[i][j];
    }
    return M;
}

// Scores a CSR batch of residue codes (0..19) with the reference run_on_sequence on `nthreads`
// host threads, one MSV_HMM per thread, sequences strided across threads. Only the scoring
// loop is timed (string building and profile construction are outside, as in
// benchmark_helper.hpp:20-38 where parsing is outside the timed region).
// Returns the wall seconds of the scoring loop, or -1 on a bad code.
double ref_score_codes(const char* hmm_path, const uint8_t* codes, const uint64_t* offsets, long n, int nthreads,
                       float* scores) {
    std::vector<std::string> seqs(n);
    for (long s = 0; s < n; ++s) {
        std::string q = "#";
        q.reserve(offsets[s + 1] - offsets[s] + 1);
        for (uint64_t k = offsets[s]; k < offsets[s + 1]; ++k) {
            if (codes[k] >= 20) return -1.0;
            q += kLetters[codes[k]];
        }
        seqs[s] = std::move(q);
    }
    if (nthreads < 1) nthreads = 1;
    auto hmm = Profile_HMM(hmm_path);
    std::vector<std::unique_ptr<MSV_HMM>> engines;
    for (int t = 0; t < nthreads; ++t) engines.emplace_back(std::make_unique<MSV_HMM>(hmm));

    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int t = 0; t < nthreads; ++t) {
        pool.emplace_back([&, t] {
            for (long s = t; s < n; s += nthreads) scores[s] = engines[t]->run_on_sequence(seqs[s]);
        });
    }
    for (auto& th : pool) th.join();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

} // extern "C"
