// msv_hmm.hpp -- C++ host surface of the MI355X MSV engine, mirroring the reference classes
// (drop-in names, argument meaning and layouts) on top of the C-ABI in msv.h:
//
//   Profile_HMM               data_readers/Profile_HMM.hpp:21-49
//   FASTA_protein_sequences   data_readers/FASTA_protein_sequences.hpp:9-14
//   MSV_HMM                   algorithms/MSV_HMM.hpp:17-44
//   Viterbi_HMM               (new) the Viterbi stage over the parts of Profile_HMM the
//                             reference parses and never scores with (Profile_HMM.cpp:107-120)
//
// Differences from the reference, all deliberate:
//   * errors throw (msv_error, or std::out_of_range for a residue outside the 20 amino acids,
//     exactly what the reference's amino_acid_num.at throws, MSV_HMM.cpp:101) instead of printing
//     and continuing with a half-built object (Profile_HMM.cpp:50-53, MSV_HMM.cpp:198-203);
//   * run_on_sequence is, as in the reference, the sequential CPU DP (this library's own
//     restatement, two rolling rows); parallel_run_on_sequence and score_batch* score on the GPU.
//     Both are bit-identical to the reference's CPU DP, so the reference's seq-vs-par differential
//     (test_MSV.cpp:23-26) compares CPU and GPU;
//   * score_batch adds the batch API the reference lacks: one kernel launch per batch.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "msv.h"

constexpr int NUM_OF_AMINO_ACIDS = 20;
constexpr int NUM_OF_TRANSITIONS = 7;

using Probability = float;
using Profile_name = std::string;
template <int N>
using Probabilities_array = std::array<Probability, N>;
template <int N>
using Probabilities_arrays_vector = std::vector<Probabilities_array<N>>;

using Protein_sequence = std::string;  // '#' sentinel + residues, as the reference
using Protein_sequences = std::vector<Protein_sequence>;
using Log_score = float;

class msv_error : public std::runtime_error {
  public:
    msv_error(msv_status s, const std::string& what) : std::runtime_error(what), status(s) {}
    msv_status status;
};

class Profile_HMM {
  public:
    explicit Profile_HMM(const std::string& file_path);

    Profile_name name;
    Probabilities_arrays_vector<NUM_OF_AMINO_ACIDS> match_emissions;
    Probabilities_arrays_vector<NUM_OF_AMINO_ACIDS> insert_emissions;
    Probabilities_arrays_vector<NUM_OF_TRANSITIONS> transitions;
    size_t model_length = 0;

    float stats_local_msv_mu = 0, stats_local_msv_lambda = 0;
    float stats_local_viterbi_mu = 0, stats_local_viterbi_lambda = 0;
    float stats_local_forward_theta = 0, stats_local_forward_lambda = 0;
};

// Residues packed for the device: codes 0..19 (255 = a symbol the scorer rejects), CSR offsets.
struct Packed_sequences {
    std::vector<uint8_t> codes;
    std::vector<uint64_t> offsets{0};
    size_t size() const { return offsets.size() - 1; }
    // '#'-prefixed strings -> codes; throws std::out_of_range on a symbol outside the 20
    static Packed_sequences pack(const Protein_sequences& seqs);
};

class FASTA_protein_sequences {
  public:
    explicit FASTA_protein_sequences(const std::string& file_path);

    Protein_sequences sequences;  // same records as the reference parser, '#'-prefixed
    Packed_sequences packed;      // the same records as device-ready codes
    std::vector<std::string> headers;
    size_t rejected = 0;
};

// A FASTA file parsed on the GPU (msv_fasta_read_device): the same records, left in device memory.
class FASTA_device {
  public:
    explicit FASTA_device(const std::string& file_path, int device = 0);
    ~FASTA_device();
    FASTA_device(const FASTA_device&) = delete;
    FASTA_device& operator=(const FASTA_device&) = delete;
    size_t size() const { return msv_fasta_device_count(handle_); }
    size_t rejected() const { return msv_fasta_device_rejected(handle_); }
    const msv_fasta_device* handle() const { return handle_; }

  private:
    msv_fasta_device* handle_ = nullptr;
};

class MSV_HMM {
  public:
    explicit MSV_HMM(const Profile_HMM& base_hmm, int device = 0);
    ~MSV_HMM();
    MSV_HMM(const MSV_HMM&) = delete;
    MSV_HMM& operator=(const MSV_HMM&) = delete;
    MSV_HMM(MSV_HMM&& o) noexcept;
    MSV_HMM& operator=(MSV_HMM&& o) noexcept;

    // One sequence ('#' + residues).  run_on_sequence: the sequential CPU DP (MSV_HMM.cpp:74-113);
    // parallel_run_on_sequence: the fused gfx950 kernel, as a batch of one (MSV_HMM.cpp:269-430).
    Log_score run_on_sequence(const Protein_sequence& seq);
    Log_score parallel_run_on_sequence(const Protein_sequence& seq, bool should_specialize = false);

    // The batch hot path: one launch for the whole set.
    std::vector<Log_score> score_batch(const Protein_sequences& seqs);
    std::vector<Log_score> score_batch(const Packed_sequences& packed);
    std::vector<Log_score> score_batch(const uint8_t* codes, const uint64_t* offsets, size_t n);
    std::vector<Log_score> score_batch(const FASTA_device& fasta);  // GPU-parsed, scored in place

    // Profiles x sequences grid (benchmark_MSV.cpp:12-24,31-41 as one call): result[p][s].
    static std::vector<std::vector<Log_score>> score_grid(const std::vector<MSV_HMM*>& profiles,
                                                          const Protein_sequences& seqs);
    // One batch sharded over several devices (profiles[k] = this model on device k), input order.
    static std::vector<Log_score> score_batch_multi(const std::vector<MSV_HMM*>& per_device,
                                                    const Protein_sequences& seqs);

    // One batch over several devices of this process, scores gathered over RCCL (msv_multi_*).
    class Multi_device;

    msv_profile* handle() { return profile_; }
    size_t model_length() const { return model_length_; }
    const std::vector<float>& emission_scores() const { return emission_scores_; }
    float tr_B_Mk() const { return tr_B_Mk_; }
    float tr_E_C() const { return tr_E_C_; }
    float tr_E_J() const { return tr_E_J_; }

  private:
    size_t model_length_ = 0;
    std::vector<float> emission_scores_;  // [20][model_length], MSV_HMM.hpp:27-28
    float tr_B_Mk_ = 0, tr_E_C_ = 0, tr_E_J_ = 0;
    msv_profile* profile_ = nullptr;
};

// MSV_HMM::Multi_device: the same model on DISTINCT devices (per_device[k] on device k), one RCCL
// communicator per device; score_batch shards the batch by residues and gathers the scores on the
// first device over RCCL (msv_multi_create / msv_multi_score_batch).  Holds the MSV_HMMs by pointer.
class MSV_HMM::Multi_device {
  public:
    explicit Multi_device(const std::vector<MSV_HMM*>& per_device);
    ~Multi_device();
    Multi_device(const Multi_device&) = delete;
    Multi_device& operator=(const Multi_device&) = delete;
    std::vector<Log_score> score_batch(const Protein_sequences& seqs);
    std::vector<Log_score> score_batch(const Packed_sequences& packed);

  private:
    msv_multi* multi_ = nullptr;
};

// The Viterbi stage (recurrence and conventions in msv.h): HMMER3's generic local Viterbi over
// the reference's parse -- insert emissions and the 7 transitions per node -- with the MSV path's specials.
// Same shape as MSV_HMM: run_on_sequence is this library's serial CPU DP, parallel_run_on_sequence and
// score_batch the gfx950 kernel (bit-identical to each other).  STATS LOCAL VITERBI gives the P-values.
class Viterbi_HMM {
  public:
    explicit Viterbi_HMM(const Profile_HMM& base_hmm, int device = 0, msv_insert_mode inserts = MSV_INSERTS_ZERO);
    ~Viterbi_HMM();
    Viterbi_HMM(const Viterbi_HMM&) = delete;
    Viterbi_HMM& operator=(const Viterbi_HMM&) = delete;
    Viterbi_HMM(Viterbi_HMM&& o) noexcept;
    Viterbi_HMM& operator=(Viterbi_HMM&& o) noexcept;

    Log_score run_on_sequence(const Protein_sequence& seq);
    Log_score parallel_run_on_sequence(const Protein_sequence& seq);
    std::vector<Log_score> score_batch(const Protein_sequences& seqs);
    std::vector<Log_score> score_batch(const Packed_sequences& packed);

    msv_vit_profile* handle() { return profile_; }
    size_t model_length() const { return model_length_; }
    float viterbi_mu = 0, viterbi_lambda = 0;  // STATS LOCAL VITERBI (Profile_HMM.cpp:86-87)

  private:
    size_t model_length_ = 0;
    bool inserts_ = false;
    std::vector<float> match_scores_, insert_scores_, transition_scores_;  // [20][M], [20][M], [M][7]
    float tr_B_Mk_ = 0, tr_E_C_ = 0, tr_E_J_ = 0;
    msv_vit_profile* profile_ = nullptr;
};

// HMMER3's filter cascade on the GPU (msv_vit_filter_batch): MSV scores of every sequence, the survivors of
// P <= F1 against (msv_mu, msv_lambda) -- a Profile_HMM's stats_local_msv_mu/lambda -- and their Viterbi
// scores (-inf where a sequence did not pass).
struct Filter_result {
    std::vector<Log_score> msv_scores;
    std::vector<uint8_t> passed;
    std::vector<Log_score> viterbi_scores;
    size_t n_passed = 0;
};
Filter_result filter_pipeline(MSV_HMM& msv, Viterbi_HMM& vit, const Packed_sequences& packed, float msv_mu,
                              float msv_lambda, double F1 = 0.02);
