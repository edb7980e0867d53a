// msv_hmm.cpp -- MSV_HMM, the reference's class surface (algorithms/MSV_HMM.hpp:17-44), on the
// C-ABI device path.  The host precompute is the reference's (MSV_HMM.cpp:35-57, host libm).
// parallel_run_on_sequence and every batch entry score on the fused gfx950 kernel; run_on_sequence
// is, as in the reference, the sequential CPU DP (the seq-vs-par differential of test_MSV.cpp).
#include <algorithm>
#include <cmath>
#include <limits>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "host_cpu.h"
#include "msv.h"
#include "msv_hmm.hpp"

namespace {

void check(msv_status s, const char* what) {
    if (s != MSV_OK) throw msv_error(s, std::string(what) + ": " + msv_status_string(s));
}

// background_frequencies, MSV_HMM.cpp:21-27
constexpr float kBackground[NUM_OF_AMINO_ACIDS] = {
    0.0787945f, 0.0151600f, 0.0535222f, 0.0668298f, 0.0397062f, 0.0695071f, 0.0229198f,
    0.0590092f, 0.0594422f, 0.0963728f, 0.0237718f, 0.0414386f, 0.0482904f, 0.0395639f,
    0.0540978f, 0.0683364f, 0.0540687f, 0.0673417f, 0.0114135f, 0.0304133f};

}  // namespace

MSV_HMM::MSV_HMM(const Profile_HMM& base_hmm, int device) : model_length_(base_hmm.model_length) {
    // MSV_HMM.cpp:38-45: [20][model_length] log-odds, column 0 = log(0) = -inf
    emission_scores_.assign(NUM_OF_AMINO_ACIDS * model_length_, 0.f);
    for (size_t i = 0; i < model_length_; ++i)
        for (size_t j = 0; j < NUM_OF_AMINO_ACIDS; ++j)
            emission_scores_[j * model_length_ + i] = std::log(base_hmm.match_emissions[i][j] / kBackground[j]);
    constexpr float nu = 2.0;  // MSV_HMM.cpp:49
    tr_B_Mk_ = std::log(2.0f / static_cast<float>(base_hmm.model_length * (base_hmm.model_length + 1)));
    tr_E_C_ = std::log((nu - 1.0f) / nu);
    tr_E_J_ = std::log(1.0f / nu);
    check(msv_profile_create(device, emission_scores_.data(), static_cast<uint32_t>(model_length_), tr_B_Mk_,
                             tr_E_C_, tr_E_J_, &profile_),
          "msv_profile_create");
}

MSV_HMM::~MSV_HMM() { msv_profile_destroy(profile_); }

MSV_HMM::MSV_HMM(MSV_HMM&& o) noexcept
    : model_length_(o.model_length_),
      emission_scores_(std::move(o.emission_scores_)),
      tr_B_Mk_(o.tr_B_Mk_),
      tr_E_C_(o.tr_E_C_),
      tr_E_J_(o.tr_E_J_),
      profile_(std::exchange(o.profile_, nullptr)) {}

MSV_HMM& MSV_HMM::operator=(MSV_HMM&& o) noexcept {
    if (this != &o) {
        msv_profile_destroy(profile_);
        model_length_ = o.model_length_;
        emission_scores_ = std::move(o.emission_scores_);
        tr_B_Mk_ = o.tr_B_Mk_;
        tr_E_C_ = o.tr_E_C_;
        tr_E_J_ = o.tr_E_J_;
        profile_ = std::exchange(o.profile_, nullptr);
    }
    return *this;
}

Log_score MSV_HMM::run_on_sequence(const Protein_sequence& seq) {
    // The reference's sequential CPU recurrence (MSV_HMM.cpp:74-113), msv_host::run_on_sequence.
    const size_t L = seq.empty() ? 0 : seq.size() - 1;  // '#' sentinel (FASTA_protein_sequences.cpp:19-20)
    std::vector<uint8_t> codes(L);
    if (L && msv_encode_residues(seq.data() + 1, L, codes.data()) != MSV_OK)
        throw std::out_of_range("residue outside the 20 amino acids");  // amino_acid_num.at, MSV_HMM.cpp:101
    return msv_host::run_on_sequence(emission_scores_.data(), model_length_, tr_B_Mk_, tr_E_C_, tr_E_J_, codes.data(),
                                     L);
}

Log_score MSV_HMM::parallel_run_on_sequence(const Protein_sequence& seq, bool /*should_specialize*/) {
    // The reference's should_specialize bakes sizes and transition constants into the OpenCL
    // program through -D defines (MSV_HMM.cpp:322-337); here the sizes are always compile-time
    // template parameters of the kernel and the constants are exact floats, so both settings
    // run the same specialised kernel and return the same (reference-exact) score.
    return score_batch(Protein_sequences{seq})[0];
}

std::vector<Log_score> MSV_HMM::score_batch(const Protein_sequences& seqs) {
    return score_batch(Packed_sequences::pack(seqs));
}

std::vector<Log_score> MSV_HMM::score_batch(const Packed_sequences& packed) {
    return score_batch(packed.codes.data(), packed.offsets.data(), packed.size());
}

std::vector<std::vector<Log_score>> MSV_HMM::score_grid(const std::vector<MSV_HMM*>& profiles,
                                                        const Protein_sequences& seqs) {
    std::vector<msv_profile*> handles;
    for (MSV_HMM* m : profiles) handles.push_back(m->profile_);
    const Packed_sequences packed = Packed_sequences::pack(seqs);
    const size_t n = packed.size();
    std::vector<Log_score> flat(handles.size() * n);
    const msv_status s = msv_score_grid(handles.data(), static_cast<uint32_t>(handles.size()), packed.codes.data(),
                                        packed.offsets.data(), n, flat.data(), nullptr);
    if (s == MSV_ERR_BAD_RESIDUE) throw std::out_of_range("residue outside the 20 amino acids");
    check(s, "msv_score_grid");
    std::vector<std::vector<Log_score>> out(handles.size());
    for (size_t p = 0; p < handles.size(); ++p) out[p].assign(flat.begin() + p * n, flat.begin() + (p + 1) * n);
    return out;
}

std::vector<Log_score> MSV_HMM::score_batch_multi(const std::vector<MSV_HMM*>& per_device,
                                                  const Protein_sequences& seqs) {
    std::vector<msv_profile*> handles;
    for (MSV_HMM* m : per_device) handles.push_back(m->profile_);
    const Packed_sequences packed = Packed_sequences::pack(seqs);
    std::vector<Log_score> out(packed.size());
    const msv_status s = msv_score_batch_multi(handles.data(), static_cast<uint32_t>(handles.size()),
                                               packed.codes.data(), packed.offsets.data(), packed.size(), out.data());
    if (s == MSV_ERR_BAD_RESIDUE) throw std::out_of_range("residue outside the 20 amino acids");
    check(s, "msv_score_batch_multi");
    return out;
}

FASTA_device::FASTA_device(const std::string& file_path, int device) {
    const msv_status s = msv_fasta_read_device(device, file_path.c_str(), nullptr, &handle_);
    if (s != MSV_OK) throw msv_error(s, std::string(msv_status_string(s)) + ": " + file_path);
}

FASTA_device::~FASTA_device() { msv_fasta_device_destroy(handle_); }

std::vector<Log_score> MSV_HMM::score_batch(const FASTA_device& fasta) {
    std::vector<Log_score> out(fasta.size());
    const msv_status s = msv_score_fasta_device(profile_, fasta.handle(), out.data());
    if (s == MSV_ERR_BAD_RESIDUE) throw std::out_of_range("residue outside the 20 amino acids");
    check(s, "msv_score_fasta_device");
    return out;
}

std::vector<Log_score> MSV_HMM::score_batch(const uint8_t* codes, const uint64_t* offsets, size_t n) {
    std::vector<Log_score> out(n);
    const msv_status s = msv_score_batch(profile_, codes, offsets, n, out.data(), nullptr);
    if (s == MSV_ERR_BAD_RESIDUE) throw std::out_of_range("residue outside the 20 amino acids");
    check(s, "msv_score_batch");
    return out;
}

MSV_HMM::Multi_device::Multi_device(const std::vector<MSV_HMM*>& per_device) {
    std::vector<msv_profile*> handles;
    for (MSV_HMM* m : per_device) handles.push_back(m->profile_);
    check(msv_multi_create(handles.data(), static_cast<uint32_t>(handles.size()), &multi_), "msv_multi_create");
}

MSV_HMM::Multi_device::~Multi_device() { msv_multi_destroy(multi_); }

std::vector<Log_score> MSV_HMM::Multi_device::score_batch(const Protein_sequences& seqs) {
    return score_batch(Packed_sequences::pack(seqs));
}

std::vector<Log_score> MSV_HMM::Multi_device::score_batch(const Packed_sequences& packed) {
    std::vector<Log_score> out(packed.size());
    const msv_status s =
        msv_multi_score_batch(multi_, packed.codes.data(), packed.offsets.data(), packed.size(), out.data());
    if (s == MSV_ERR_BAD_RESIDUE) throw std::out_of_range("residue outside the 20 amino acids");
    check(s, "msv_multi_score_batch");
    return out;
}

// ---- Viterbi stage --------------------------------------------------------------------
Viterbi_HMM::Viterbi_HMM(const Profile_HMM& base_hmm, int device, msv_insert_mode inserts)
    : viterbi_mu(base_hmm.stats_local_viterbi_mu),
      viterbi_lambda(base_hmm.stats_local_viterbi_lambda),
      model_length_(base_hmm.model_length),
      inserts_(inserts == MSV_INSERTS_LOG_ODDS) {
    const size_t M = model_length_;
    match_scores_.assign(NUM_OF_AMINO_ACIDS * M, 0.f);
    insert_scores_.assign(NUM_OF_AMINO_ACIDS * M, 0.f);
    transition_scores_.assign(NUM_OF_TRANSITIONS * M, 0.f);
    for (size_t k = 0; k < M; ++k) {
        for (size_t r = 0; r < NUM_OF_AMINO_ACIDS; ++r) {
            match_scores_[r * M + k] = std::log(base_hmm.match_emissions[k][r] / kBackground[r]);  // MSV_HMM.cpp:38-45
            if (inserts_) insert_scores_[r * M + k] = std::log(base_hmm.insert_emissions[k][r] / kBackground[r]);
        }
        for (size_t t = 0; t < NUM_OF_TRANSITIONS; ++t)
            transition_scores_[k * NUM_OF_TRANSITIONS + t] = std::log(base_hmm.transitions[k][t]);
    }
    constexpr float nu = 2.0;  // the MSV path's specials, MSV_HMM.cpp:49-53
    tr_B_Mk_ = std::log(2.0f / static_cast<float>(M * (M + 1)));
    tr_E_C_ = std::log((nu - 1.0f) / nu);
    tr_E_J_ = std::log(1.0f / nu);
    check(msv_vit_profile_create(device, match_scores_.data(), inserts_ ? insert_scores_.data() : nullptr,
                                 transition_scores_.data(), static_cast<uint32_t>(M), tr_B_Mk_, tr_E_C_, tr_E_J_,
                                 &profile_),
          "msv_vit_profile_create");
}

Viterbi_HMM::~Viterbi_HMM() { msv_vit_profile_destroy(profile_); }

Viterbi_HMM::Viterbi_HMM(Viterbi_HMM&& o) noexcept
    : viterbi_mu(o.viterbi_mu),
      viterbi_lambda(o.viterbi_lambda),
      model_length_(o.model_length_),
      inserts_(o.inserts_),
      match_scores_(std::move(o.match_scores_)),
      insert_scores_(std::move(o.insert_scores_)),
      transition_scores_(std::move(o.transition_scores_)),
      tr_B_Mk_(o.tr_B_Mk_),
      tr_E_C_(o.tr_E_C_),
      tr_E_J_(o.tr_E_J_),
      profile_(std::exchange(o.profile_, nullptr)) {}

Viterbi_HMM& Viterbi_HMM::operator=(Viterbi_HMM&& o) noexcept {
    if (this != &o) {
        msv_vit_profile_destroy(profile_);
        viterbi_mu = o.viterbi_mu;
        viterbi_lambda = o.viterbi_lambda;
        model_length_ = o.model_length_;
        inserts_ = o.inserts_;
        match_scores_ = std::move(o.match_scores_);
        insert_scores_ = std::move(o.insert_scores_);
        transition_scores_ = std::move(o.transition_scores_);
        tr_B_Mk_ = o.tr_B_Mk_;
        tr_E_C_ = o.tr_E_C_;
        tr_E_J_ = o.tr_E_J_;
        profile_ = std::exchange(o.profile_, nullptr);
    }
    return *this;
}

Log_score Viterbi_HMM::run_on_sequence(const Protein_sequence& seq) {
    const size_t L = seq.empty() ? 0 : seq.size() - 1;
    std::vector<uint8_t> codes(L);
    if (L && msv_encode_residues(seq.data() + 1, L, codes.data()) != MSV_OK)
        throw std::out_of_range("residue outside the 20 amino acids");
    return msv_host::viterbi_run_on_sequence(match_scores_.data(), inserts_ ? insert_scores_.data() : nullptr,
                                             transition_scores_.data(), model_length_, tr_B_Mk_, tr_E_C_, tr_E_J_,
                                             codes.data(), L);
}

Log_score Viterbi_HMM::parallel_run_on_sequence(const Protein_sequence& seq) {
    return score_batch(Protein_sequences{seq})[0];
}

std::vector<Log_score> Viterbi_HMM::score_batch(const Protein_sequences& seqs) {
    return score_batch(Packed_sequences::pack(seqs));
}

std::vector<Log_score> Viterbi_HMM::score_batch(const Packed_sequences& packed) {
    std::vector<Log_score> out(packed.size());
    const msv_status s = msv_vit_score_batch(profile_, packed.codes.data(), packed.offsets.data(), packed.size(),
                                             out.data(), nullptr);
    if (s == MSV_ERR_BAD_RESIDUE) throw std::out_of_range("residue outside the 20 amino acids");
    check(s, "msv_vit_score_batch");
    return out;
}

Filter_result filter_pipeline(MSV_HMM& msv, Viterbi_HMM& vit, const Packed_sequences& packed, float msv_mu,
                              float msv_lambda, double F1) {
    Filter_result r;
    const size_t n = packed.size();
    r.msv_scores.resize(n);
    r.passed.resize(n);
    r.viterbi_scores.resize(n);
    uint64_t passed = 0;
    const msv_status s = msv_vit_filter_batch(msv.handle(), vit.handle(), packed.codes.data(), packed.offsets.data(),
                                              n, msv_mu, msv_lambda, F1, r.msv_scores.data(), r.passed.data(),
                                              r.viterbi_scores.data(), &passed);
    if (s == MSV_ERR_BAD_RESIDUE) throw std::out_of_range("residue outside the 20 amino acids");
    check(s, "msv_vit_filter_batch");
    r.n_passed = static_cast<size_t>(passed);
    return r;
}
