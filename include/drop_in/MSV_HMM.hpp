// MSV_HMM.hpp -- forwarding header with the reference's file name (algorithms/MSV_HMM.hpp), so the
// reference's own callers (test_MSV.cpp:1-2, benchmark_helper.hpp:1) build UNCHANGED against this
// library: `#include "MSV_HMM.hpp"` resolves here once the reference's algorithms/MSV_HMM.{hpp,cpp}
// are removed from the build.  The classes live in ../msv_hmm.hpp.  These
// forwarding headers sit in their own directory (include/drop_in/) because MSV_HMM.hpp and msv_hmm.hpp
// would be one file on a case-insensitive file system.
#pragma once

#include "FASTA_protein_sequences.hpp"
#include "Profile_HMM.hpp"

// The reference's remaining aliases (MSV_HMM.hpp:9-15).
template <int N>
using Log_scores_array = std::array<Log_score, N>;
template <int N>
using Log_scores_arrays_vector = std::vector<Log_scores_array<N>>;
using Kernels_source_code = std::string;
