// host_cpu.h -- host-only internals shared by msv_hmm.cpp and the sanitizer drivers (host_common.cpp).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace msv_host {

// MSV_HMM::run_on_sequence (MSV_HMM.cpp:74-113) on codes 0..19: emission_scores is the [20][M]
// residue-major table of MSV_HMM.cpp:38-45 (M = LENG + 1), the score is C_L + tr_move.
float run_on_sequence(const float* emission_scores, size_t M, float tr_B_Mk, float tr_E_C, float tr_E_J,
                      const uint8_t* codes, size_t L);

// The Viterbi stage's DP (msv.h, msv_vit_cpu_score) on codes 0..19: msc / isc [20][M] (isc may be null:
// zero insert scores), tsc [M][7] log transitions.
float viterbi_run_on_sequence(const float* msc, const float* isc, const float* tsc, size_t M, float tr_B_Mk,
                              float tr_E_C, float tr_E_J, const uint8_t* codes, size_t L);

}  // namespace msv_host
