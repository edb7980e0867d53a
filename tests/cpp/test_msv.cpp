// test_msv.cpp -- GPU parity driver in the shape of the reference's differential test
// (algorithms/test_MSV.cpp:14-36): every profile x fasta_like_example.fsa, scored through
// run_on_sequence (the CPU DP), parallel_run_on_sequence(seq) and parallel_run_on_sequence(seq,
// true) (the GPU kernel), plus the batch API.  Unlike the reference (which only checks seq vs par
// within 1e-4, test_MSV.cpp:10-12,26), every score is compared BITWISE with the golden scores the
// reference's own CPU path produced (tests/golden/example_scores.tsv, oracle/make_golden.py), and
// the seq-vs-par differential itself (CPU vs GPU) runs bitwise on seeded sequences for every
// profile.
// Usage: test_msv <repo_root>   (exit 0 = pass)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "msv_hmm.hpp"

static bool same_bits(float a, float b) { return std::memcmp(&a, &b, sizeof(float)) == 0; }

int main(int argc, char** argv) {
    const std::string root = argc > 1 ? argv[1] : ".";
    std::map<std::string, std::vector<float>> golden;
    std::ifstream g(root + "/tests/golden/example_scores.tsv");
    std::string line;
    while (std::getline(g, line)) {
        if (line.empty() || line[0] == '#') continue;
        std::istringstream ss(line);
        std::string prof, idx, len, hex;
        ss >> prof >> idx >> len >> hex;
        golden[prof].push_back(std::strtof(hex.c_str(), nullptr));
    }
    if (golden.size() != 24) {
        std::printf("test_msv: expected 24 profiles in golden file, got %zu\n", golden.size());
        return 1;
    }
    auto fasta = FASTA_protein_sequences(root + "/data/FASTA_files/fasta_like_example.fsa");
    int checked = 0;
    for (const auto& [prof, want] : golden) {
        auto msv = MSV_HMM(Profile_HMM(root + "/data/profile_HMMs/" + prof));
        auto batch = msv.score_batch(fasta.sequences);
        for (size_t i = 0; i < fasta.sequences.size(); ++i) {
            const auto& protein = fasta.sequences[i];
            float seq = msv.run_on_sequence(protein);
            float par = msv.parallel_run_on_sequence(protein);
            float par_spec = msv.parallel_run_on_sequence(protein, true);
            if (!same_bits(seq, want[i]) || !same_bits(par, want[i]) || !same_bits(par_spec, want[i]) ||
                !same_bits(batch[i], want[i])) {
                std::printf("test_msv failed! %s seq %zu: golden %a, run %a, par %a, par_spec %a, batch %a\n",
                            prof.c_str(), i, want[i], seq, par, par_spec, batch[i]);
                return 1;
            }
            ++checked;
        }
    }
    // the whole grid in one call (benchmark_MSV.cpp's loop over every profile)
    {
        std::vector<MSV_HMM> engines;
        engines.reserve(golden.size());
        for (const auto& kv : golden) engines.emplace_back(Profile_HMM(root + "/data/profile_HMMs/" + kv.first));
        std::vector<MSV_HMM*> ptrs;
        for (auto& e : engines) ptrs.push_back(&e);
        auto grid = MSV_HMM::score_grid(ptrs, fasta.sequences);
        size_t p = 0;
        for (const auto& [prof, want] : golden) {
            for (size_t i = 0; i < want.size(); ++i) {
                if (!same_bits(grid[p][i], want[i])) {
                    std::printf("test_msv failed! grid %s seq %zu: golden %a, grid %a\n", prof.c_str(), i, want[i],
                                grid[p][i]);
                    return 1;
                }
                ++checked;
            }
            ++p;
        }
    }
    // the same FASTA parsed on the GPU and scored in place
    {
        auto gfa = FASTA_device(root + "/data/FASTA_files/fasta_like_example.fsa");
        for (const auto& [prof, want] : golden) {
            auto m = MSV_HMM(Profile_HMM(root + "/data/profile_HMMs/" + prof));
            auto got = m.score_batch(gfa);
            for (size_t i = 0; i < want.size(); ++i) {
                if (!same_bits(got[i], want[i])) {
                    std::printf("test_msv failed! device FASTA %s seq %zu: golden %a, got %a\n", prof.c_str(), i,
                                want[i], got[i]);
                    return 1;
                }
                ++checked;
            }
        }
    }
    // the reference's seq-vs-par differential (test_MSV.cpp:23-26), bitwise: the CPU DP against the
    // GPU kernel on seeded sequences of lengths 0..700 for every profile (one GPU batch per profile)
    {
        uint64_t x = 0x9E3779B97F4A7C15ull;
        auto next = [&] {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            return x;
        };
        const char* letters = "ACDEFGHIKLMNPQRSTVWY";
        Protein_sequences seqs;
        for (int i = 0; i < 40; ++i) {
            std::string s = "#";
            const size_t L = i < 3 ? static_cast<size_t>(i) : next() % 701;
            for (size_t k = 0; k < L; ++k) s += letters[next() % 20];
            seqs.push_back(s);
        }
        for (const auto& kv : golden) {
            const Profile_HMM prof(root + "/data/profile_HMMs/" + kv.first);
            auto m = MSV_HMM(prof);
            auto par = m.score_batch(seqs);
            for (size_t i = 0; i < seqs.size(); ++i) {
                const float seq = m.run_on_sequence(seqs[i]);
                if (!same_bits(seq, par[i])) {
                    std::printf("test_msv failed! seq vs par %s random seq %zu (L=%zu): cpu %a, gpu %a\n",
                                kv.first.c_str(), i, seqs[i].size() - 1, seq, par[i]);
                    return 1;
                }
                ++checked;
            }
            // the Viterbi stage in the same shape: CPU DP vs the gfx950 kernel, both insert modes
            for (msv_insert_mode mode : {MSV_INSERTS_ZERO, MSV_INSERTS_LOG_ODDS}) {
                auto v = Viterbi_HMM(prof, 0, mode);
                auto vpar = v.score_batch(seqs);
                for (size_t i = 0; i < seqs.size(); ++i) {
                    const float seq = v.run_on_sequence(seqs[i]);
                    if (!same_bits(seq, vpar[i])) {
                        std::printf("test_msv failed! Viterbi seq vs par %s (inserts %d) seq %zu: cpu %a, gpu %a\n",
                                    kv.first.c_str(), static_cast<int>(mode), i, seq, vpar[i]);
                        return 1;
                    }
                    ++checked;
                }
            }
        }
    }
    // the filter cascade: MSV -> P <= F1 -> Viterbi on the survivors, against the pieces one by one
    {
        const Profile_HMM prof(root + "/data/profile_HMMs/1400.hmm");
        auto m = MSV_HMM(prof);
        auto v = Viterbi_HMM(prof);
        const Packed_sequences packed = Packed_sequences::pack(fasta.sequences);
        const Filter_result r = filter_pipeline(m, v, packed, prof.stats_local_msv_mu, prof.stats_local_msv_lambda, 1.0);
        const auto want_m = m.score_batch(packed);
        const auto want_v = v.score_batch(packed);
        for (size_t i = 0; i < packed.size(); ++i)
            if (!same_bits(r.msv_scores[i], want_m[i]) || !r.passed[i] || !same_bits(r.viterbi_scores[i], want_v[i])) {
                std::printf("test_msv failed! filter_pipeline seq %zu\n", i);
                return 1;
            }
        if (r.n_passed != packed.size()) {
            std::printf("test_msv failed! filter_pipeline F1 = 1 passed %zu of %zu\n", r.n_passed, packed.size());
            return 1;
        }
        checked += static_cast<int>(2 * packed.size());
    }
    // one device through the RCCL multi-device context (1-rank communicator; the shard's scores take
    // the self send/recv path of the gather) equals one launch
    {
        auto m = MSV_HMM(Profile_HMM(root + "/data/profile_HMMs/1400.hmm"));
        MSV_HMM::Multi_device multi({&m});
        auto got = multi.score_batch(fasta.sequences);
        auto want = m.score_batch(fasta.sequences);
        for (size_t i = 0; i < want.size(); ++i)
            if (!same_bits(got[i], want[i])) {
                std::printf("test_msv failed! RCCL multi-device seq %zu: %a vs %a\n", i, got[i], want[i]);
                return 1;
            }
        checked += static_cast<int>(want.size());
    }
    // page-locked buffers from msv_host_alloc: residues read in place by the kernel, scores written by it
    // (the FFI caller's zero-copy path) -- equal to the pageable path
    {
        auto m = MSV_HMM(Profile_HMM(root + "/data/profile_HMMs/1400.hmm"));
        const size_t n = fasta.sequences.size();
        std::vector<uint8_t> codes;
        std::vector<uint64_t> offs(1, 0);
        for (const auto& s : fasta.sequences) {  // '#' + residues, as the reference stores them
            std::vector<uint8_t> c(s.size() - 1);
            if (msv_encode_residues(s.c_str() + 1, s.size() - 1, c.data()) != MSV_OK) return 1;
            codes.insert(codes.end(), c.begin(), c.end());
            offs.push_back(codes.size());
        }
        void *pc = nullptr, *ps = nullptr;
        if (msv_host_alloc(codes.size(), &pc) != MSV_OK || msv_host_alloc(n * sizeof(float), &ps) != MSV_OK) {
            std::printf("test_msv failed! msv_host_alloc\n");
            return 1;
        }
        std::memcpy(pc, codes.data(), codes.size());
        std::vector<float> want(n);
        if (msv_score_batch(m.handle(), codes.data(), offs.data(), n, want.data(), nullptr) != MSV_OK ||
            msv_score_batch(m.handle(), static_cast<uint8_t*>(pc), offs.data(), n, static_cast<float*>(ps),
                            nullptr) != MSV_OK) {
            std::printf("test_msv failed! msv_score_batch on pinned buffers\n");
            return 1;
        }
        for (size_t i = 0; i < n; ++i)
            if (!same_bits(static_cast<float*>(ps)[i], want[i])) {
                std::printf("test_msv failed! pinned seq %zu: %a vs %a\n", i, static_cast<float*>(ps)[i], want[i]);
                return 1;
            }
        msv_host_free(pc);
        msv_host_free(ps);
        checked += static_cast<int>(n);
    }
    // error behaviour: a residue outside the 20 throws std::out_of_range like amino_acid_num.at
    auto msv = MSV_HMM(Profile_HMM(root + "/data/profile_HMMs/100.hmm"));
    bool threw = false;
    try {
        msv.run_on_sequence("#ACDXEF");
    } catch (const std::out_of_range&) {
        threw = true;
    }
    try {
        msv.parallel_run_on_sequence("#ACDXEF");
        threw = false;
    } catch (const std::out_of_range&) {
    }
    if (!threw) {
        std::printf("test_msv failed! bad residue did not throw\n");
        return 1;
    }
    if (!std::isinf(msv.run_on_sequence("#")) || msv.run_on_sequence("#") > 0 ||
        !std::isinf(msv.parallel_run_on_sequence("#")) || msv.parallel_run_on_sequence("#") > 0) {
        std::printf("test_msv failed! empty sequence must score -inf\n");
        return 1;
    }
    std::printf("test_msv passed: %d scores bit-exact\n", checked);
    return 0;
}
