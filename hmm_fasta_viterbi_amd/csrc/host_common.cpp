// host_common.cpp -- the host-only part of the C-ABI (include/msv.h): status strings, the
// reference's per-sequence transitions and precompute (MSV_HMM.cpp:35-64), residue-balanced
// shard bounds, and the sequential CPU DP behind MSV_HMM::run_on_sequence (MSV_HMM.cpp:74-113).
// No HIP in this translation unit, so it and host_parsers.cpp also build as a plain-g++
// sanitizer target (csrc/Makefile `asan`, `tsan`) with no device present.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

#include "host_cpu.h"
#include "msv.h"

extern "C" {

const char* msv_status_string(msv_status s) {
    switch (s) {
        case MSV_OK: return "MSV_OK";
        case MSV_ERR_INVALID_ARGUMENT: return "MSV_ERR_INVALID_ARGUMENT";
        case MSV_ERR_IO: return "MSV_ERR_IO";
        case MSV_ERR_PARSE: return "MSV_ERR_PARSE";
        case MSV_ERR_BAD_RESIDUE: return "MSV_ERR_BAD_RESIDUE";
        case MSV_ERR_SEQUENCE_TOO_LONG: return "MSV_ERR_SEQUENCE_TOO_LONG";
        case MSV_ERR_UNSUPPORTED_MODEL: return "MSV_ERR_UNSUPPORTED_MODEL";
        case MSV_ERR_NO_DEVICE: return "MSV_ERR_NO_DEVICE";
        case MSV_ERR_HIP: return "MSV_ERR_HIP";
        case MSV_ERR_OUT_OF_MEMORY: return "MSV_ERR_OUT_OF_MEMORY";
        case MSV_ERR_RCCL: return "MSV_ERR_RCCL";
    }
    return "MSV_ERR_UNKNOWN";
}

const char* msv_version(void) { return "msv-mi355x 0.1.0 (gfx950)"; }

void msv_sequence_transitions(uint64_t L, float* tr_loop, float* tr_move) {
    // MSV_HMM.cpp:59-64: size = seq.size() - 1; log(size / float(size + 3)), log(3 / float(size + 3))
    const uint64_t size = L;
    *tr_loop = std::log(size / static_cast<float>(size + 3));
    *tr_move = std::log(3 / static_cast<float>(size + 3));
}

msv_status msv_hmm_msv_scores(const msv_hmm* hmm, float* emission_scores, float* tr_B_Mk, float* tr_E_C,
                              float* tr_E_J) {
    if (!hmm || !emission_scores || !tr_B_Mk || !tr_E_C || !tr_E_J) return MSV_ERR_INVALID_ARGUMENT;
    // MSV_HMM::MSV_HMM, MSV_HMM.cpp:35-57
    static constexpr float bg[20] = {0.0787945f, 0.0151600f, 0.0535222f, 0.0668298f, 0.0397062f,
                                     0.0695071f, 0.0229198f, 0.0590092f, 0.0594422f, 0.0963728f,
                                     0.0237718f, 0.0414386f, 0.0482904f, 0.0395639f, 0.0540978f,
                                     0.0683364f, 0.0540687f, 0.0673417f, 0.0114135f, 0.0304133f};
    const size_t M = msv_hmm_model_length(hmm);
    const float* match = msv_hmm_match_emissions(hmm);
    for (size_t i = 0; i < M; ++i)
        for (size_t j = 0; j < 20; ++j) emission_scores[j * M + i] = std::log(match[i * 20 + j] / bg[j]);
    constexpr float nu = 2.0f;
    *tr_B_Mk = std::log(2.0f / static_cast<float>(M * (M + 1)));
    *tr_E_C = std::log((nu - 1.0f) / nu);
    *tr_E_J = std::log(1.0f / nu);
    return MSV_OK;
}

msv_status msv_hmm_viterbi_scores(const msv_hmm* hmm, int insert_mode, float* match_scores, float* insert_scores,
                                  float* transition_scores, float* tr_B_Mk, float* tr_E_C, float* tr_E_J) {
    if (!hmm || (insert_mode != MSV_INSERTS_ZERO && insert_mode != MSV_INSERTS_LOG_ODDS))
        return MSV_ERR_INVALID_ARGUMENT;
    const size_t M = msv_hmm_model_length(hmm);
    std::vector<float> msc(20 * M);
    float b, c, j;
    msv_status s = msv_hmm_msv_scores(hmm, msc.data(), &b, &c, &j);  // match scores and specials: the MSV path's
    if (s != MSV_OK) return s;
    if (match_scores) std::copy(msc.begin(), msc.end(), match_scores);
    if (insert_scores) {
        static constexpr float bg[20] = {0.0787945f, 0.0151600f, 0.0535222f, 0.0668298f, 0.0397062f,
                                         0.0695071f, 0.0229198f, 0.0590092f, 0.0594422f, 0.0963728f,
                                         0.0237718f, 0.0414386f, 0.0482904f, 0.0395639f, 0.0540978f,
                                         0.0683364f, 0.0540687f, 0.0673417f, 0.0114135f, 0.0304133f};
        const float* ins = msv_hmm_insert_emissions(hmm);  // Profile_HMM.cpp:113-115
        for (size_t k = 0; k < M; ++k)
            for (size_t r = 0; r < 20; ++r)
                insert_scores[r * M + k] = insert_mode == MSV_INSERTS_LOG_ODDS ? std::log(ins[k * 20 + r] / bg[r]) : 0.0f;
    }
    if (transition_scores) {
        const float* t = msv_hmm_transitions(hmm);  // p = exp(-x) as parsed (Profile_HMM.cpp:41, :116-119)
        for (size_t k = 0; k < M * 7; ++k) transition_scores[k] = std::log(t[k]);
    }
    if (tr_B_Mk) *tr_B_Mk = b;
    if (tr_E_C) *tr_E_C = c;
    if (tr_E_J) *tr_E_J = j;
    return MSV_OK;
}

msv_status msv_vit_cpu_score(const float* match_scores, const float* insert_scores, const float* transition_scores,
                             uint32_t model_length, float tr_B_Mk, float tr_E_C, float tr_E_J, const uint8_t* codes,
                             uint64_t L, float* score) {
    if (!match_scores || !transition_scores || !score || model_length < 2 || (L && !codes))
        return MSV_ERR_INVALID_ARGUMENT;
    for (uint64_t i = 0; i < L; ++i)
        if (codes[i] >= 20) return MSV_ERR_BAD_RESIDUE;
    *score = msv_host::viterbi_run_on_sequence(match_scores, insert_scores, transition_scores, model_length, tr_B_Mk,
                                               tr_E_C, tr_E_J, codes, L);
    return MSV_OK;
}

msv_status msv_shard_bounds(const uint64_t* offsets, uint64_t n, uint32_t n_shards, uint64_t* bounds) {
    if (!bounds || n_shards == 0 || (n && !offsets)) return MSV_ERR_INVALID_ARGUMENT;
    bounds[0] = 0;
    bounds[n_shards] = n;
    if (n == 0) {
        for (uint32_t k = 1; k < n_shards; ++k) bounds[k] = 0;
        return MSV_OK;
    }
    const uint64_t total = offsets[n] - offsets[0];
    for (uint32_t k = 1; k < n_shards; ++k) {
        // first sequence whose END reaches the k-th residue quantile (np.searchsorted(offsets[1:], t, 'left'))
        const unsigned __int128 q = static_cast<unsigned __int128>(total) * k / n_shards;
        const uint64_t target = offsets[0] + static_cast<uint64_t>(q);
        bounds[k] = static_cast<uint64_t>(std::lower_bound(offsets + 1, offsets + 1 + n, target) - (offsets + 1));
    }
    for (uint32_t k = 1; k <= n_shards; ++k) bounds[k] = std::min(n, std::max(bounds[k], bounds[k - 1]));
    return MSV_OK;
}

}  // extern "C"

namespace msv_host {

float run_on_sequence(const float* emission_scores, size_t M, float tr_B_Mk, float tr_E_C, float tr_E_J,
                      const uint8_t* codes, size_t L) {
    // The reference's sequential CPU recurrence (MSV_HMM.cpp:74-113) over two rolling rows instead
    // of the (L+1) x (M+5) matrix.  Same IEEE float ops in the same order and std::max argument
    // order: Bt = B' + tr_B_Mk, M_j = e[r][j] + max(M'_{j-1}, Bt), then J, C, N, B from the new E.
    // Only E is reduced in a different order: max is exact, and the sign of a zero E never reaches
    // a score (E only enters E + tr_E_J / E + tr_E_C with nonzero constants).  Codes must be < 20.
    constexpr float ninf = -std::numeric_limits<float>::infinity();
    float loop, move;
    msv_sequence_transitions(L, &loop, &move);  // init_transitions_depend_on_seq, MSV_HMM.cpp:59-64
    std::vector<float> prev(M, ninf), cur(M, ninf);  // [0] = the dummy M0 column, -inf on every row
    float J = ninf, C = ninf, N = 0.0f, B = move;    // row 0 (MSV_HMM.cpp:86,96-97)
    for (size_t i = 0; i < L; ++i) {
        const float* e = emission_scores + static_cast<size_t>(codes[i]) * M;
        const float Bt = B + tr_B_Mk;
        const float* pv = prev.data();
        float* cv = cur.data();
        for (size_t j = 1; j < M; ++j) cv[j] = e[j] + std::max(pv[j - 1], Bt);
        float Ek[8] = {ninf, ninf, ninf, ninf, ninf, ninf, ninf, ninf};
        size_t j = 1;
        for (; j + 8 <= M; j += 8)
            for (int q = 0; q < 8; ++q) Ek[q] = std::max(Ek[q], cv[j + q]);
        for (; j < M; ++j) Ek[0] = std::max(Ek[0], cv[j]);
        float E = ninf;
        for (float x : Ek) E = std::max(E, x);
        J = std::max(J + loop, E + tr_E_J);
        C = std::max(C + loop, E + tr_E_C);
        N = N + loop;
        B = std::max(N + move, J + move);
        std::swap(prev, cur);
    }
    return C + move;  // dp.back()[C] + tr_move; -inf for an empty sequence
}

float viterbi_run_on_sequence(const float* msc, const float* isc, const float* tsc, size_t M, float tr_B_Mk,
                              float tr_E_C, float tr_E_J, const uint8_t* codes, size_t L) {
    // The Viterbi stage's sequential DP (msv.h): HMMER3's generic local Viterbi over the reference's parse
    // with the MSV specials.  One row of each state, updated in place from the highest node down (M(k)
    // and I(k) read only the previous row at k-1 and k), then the row's D chain from the lowest node up.
    // Nodes K = M - 1; transitions of node t at tsc[t * 7 + x], read for nodes 1 .. K-1 only.
    constexpr float ninf = -std::numeric_limits<float>::infinity();
    enum { MM, MI, MD, IM, II, DM, DD };
    const size_t K = M - 1;
    float loop, move;
    msv_sequence_transitions(L, &loop, &move);
    std::vector<float> Mv(M, ninf), Iv(M, ninf), Dv(M, ninf);  // [0]: the dummy column, -inf on every row
    float J = ninf, C = ninf, N = 0.0f, B = move;
    for (size_t i = 0; i < L; ++i) {
        const size_t r = codes[i];
        const float* ms = msc + r * M;
        const float* is = isc ? isc + r * M : nullptr;
        const float Bt = B + tr_B_Mk;
        float E = ninf;
        for (size_t k = K; k >= 1; --k) {
            const float* tp = tsc + (k - 1) * 7;  // into node k from node k-1
            if (k < K) {
                const float* tk = tsc + k * 7;
                const float iv = std::max(Mv[k] + tk[MI], Iv[k] + tk[II]);
                Iv[k] = is ? iv + is[k] : iv;
            } else {
                Iv[k] = ninf;  // no insert state at node K
            }
            float m = Bt;
            if (k > 1) m = std::max(std::max(Mv[k - 1] + tp[MM], Iv[k - 1] + tp[IM]), std::max(Dv[k - 1] + tp[DM], m));
            Mv[k] = m + ms[k];
            E = std::max(E, Mv[k]);
        }
        Dv[1] = ninf;  // entered from node 0, which only B leaves
        for (size_t k = 2; k <= K; ++k) {
            const float* tp = tsc + (k - 1) * 7;
            Dv[k] = std::max(Mv[k - 1] + tp[MD], Dv[k - 1] + tp[DD]);
        }
        E = std::max(E, Dv[K]);
        J = std::max(J + loop, E + tr_E_J);
        C = std::max(C + loop, E + tr_E_C);
        N = N + loop;
        B = std::max(N + move, J + move);
    }
    return C + move;
}

}  // namespace msv_host
