/*
 * msv_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C restatement of the reference's MSV CPU path (IvanTyulyandin/HMM_FASTA_Viterbi):
 *   - HMMER3 profile parsing           data_readers/Profile_HMM.cpp:8-122
 *   - FASTA parsing + residue filter   data_readers/FASTA_protein_sequences.cpp:9-44
 *   - MSV host precompute              algorithms/MSV_HMM.cpp:35-57
 *   - per-sequence transitions         algorithms/MSV_HMM.cpp:59-64
 *   - the MSV dynamic programme        algorithms/MSV_HMM.cpp:74-113
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this file's
 * shared object.  The product (hmm_fasta_viterbi_amd/, libmsv_hip.so) never links it.
 *
 * Parity is pinned: tests/test_oracle_golden.py checks this restatement bit-for-bit against the
 * golden scores produced by the reference's own CPU path compiled from /root/reference
 * (oracle/Makefile -> oracle/_ref, oracle/make_golden.py -> tests/golden/).
 *
 * The DP is kept performance-faithful to the reference (full (L+1) x (M+5) matrix, scalar loop,
 * per-residue table lookup), because it is also the "port" CPU baseline.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NUM_AA 20
#define NUM_TR 7

/* MSV_HMM.cpp:21-27 (HMMER p7_AminoFrequencies) */
static const float background_frequencies[NUM_AA] = {
    0.0787945f, 0.0151600f, 0.0535222f, 0.0668298f, /* A C D E */
    0.0397062f, 0.0695071f, 0.0229198f, 0.0590092f, /* F G H I */
    0.0594422f, 0.0963728f, 0.0237718f, 0.0414386f, /* K L M N */
    0.0482904f, 0.0395639f, 0.0540978f, 0.0683364f, /* P Q R S */
    0.0540687f, 0.0673417f, 0.0114135f, 0.0304133f  /* T V W Y */
};

/* MSV_HMM.cpp:29-31 : alphabetical one-letter order == .hmm column order */
static const char amino_acids[NUM_AA + 1] = "ACDEFGHIKLMNPQRSTVWY";

int oracle_residue_code(char c) {
    const char* p = (c != '\0') ? strchr(amino_acids, c) : NULL;
    return p ? (int)(p - amino_acids) : -1;
}

/* ------------------------------------------------------------------------------------------ */
/* Profile HMM (Profile_HMM.hpp:21-49)                                                        */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    char name[256];
    size_t model_length; /* LENG + 1 (dummy node 0), Profile_HMM.cpp:66-71 */
    float stats_local_msv_mu, stats_local_msv_lambda;
    float stats_local_viterbi_mu, stats_local_viterbi_lambda;
    float stats_local_forward_theta, stats_local_forward_lambda;
    float* match_emissions;  /* [model_length][20], node 0 zero-filled */
    float* insert_emissions; /* [model_length][20] */
    float* transitions;      /* [model_length][7] */
} oracle_hmm;

static char* read_line(FILE* f, char** buf, size_t* cap) {
    ssize_t n = getline(buf, cap, f);
    if (n < 0) return NULL;
    if (n > 0 && (*buf)[n - 1] == '\n') (*buf)[n - 1] = '\0';
    return *buf;
}

/* skip_next_words(view, 1): Profile_HMM.cpp:10-13, without the npos UB on the last token */
static const char* skip_word(const char* s) {
    while (*s && *s != ' ') ++s;
    while (*s == ' ') ++s;
    return s;
}

/* read_value_after_tag: Profile_HMM.cpp:15-26 (prefix match on the left-stripped line) */
static int value_after_tag(FILE* f, const char* tag, char** buf, size_t* cap, const char** out) {
    size_t tl = strlen(tag);
    while (read_line(f, buf, cap)) {
        const char* s = *buf;
        while (*s == ' ') ++s;
        if (strncmp(s, tag, tl) == 0) {
            *out = skip_word(s);
            return 1;
        }
    }
    return 0;
}

/* parse_probabilities<N>: Profile_HMM.cpp:35-45 ; p = exp(-x), '*' parses as 0 -> p = 1 */
static void parse_probs(const char* s, float* out, int n) {
    while (*s == ' ') ++s;
    for (int i = 0; i < n; ++i) {
        out[i] = expf(-1 * strtof(s, NULL));
        s = skip_word(s);
    }
}

void oracle_hmm_free(oracle_hmm* h) {
    free(h->match_emissions);
    free(h->insert_emissions);
    free(h->transitions);
    memset(h, 0, sizeof(*h));
}

/* Profile_HMM::Profile_HMM: Profile_HMM.cpp:48-60. Returns 0 on success. */
int oracle_hmm_load(const char* path, oracle_hmm* h) {
    memset(h, 0, sizeof(*h));
    FILE* f = fopen(path, "r");
    if (!f) return -1;
    char* buf = NULL;
    size_t cap = 0;
    const char* v = NULL;
    int rc = -2;

    if (!value_after_tag(f, "NAME", &buf, &cap, &v)) goto out; /* :62-64 */
    snprintf(h->name, sizeof(h->name), "%s", v);
    if (!value_after_tag(f, "LENG", &buf, &cap, &v)) goto out; /* :66-71 */
    h->model_length = (size_t)atoi(v) + 1;

    for (int i = 0; i < 3; ++i) { /* :73-94 */
        if (!value_after_tag(f, "STATS", &buf, &cap, &v)) goto out;
        const char* d = skip_word(v); /* skip LOCAL */
        char kind = d[0];
        const char* nums = skip_word(d);
        char* rest = NULL;
        float a = strtof(nums, &rest);
        float b = strtof(rest, NULL);
        if (kind == 'M') { h->stats_local_msv_mu = a; h->stats_local_msv_lambda = b; }
        else if (kind == 'V') { h->stats_local_viterbi_mu = a; h->stats_local_viterbi_lambda = b; }
        else if (kind == 'F') { h->stats_local_forward_theta = a; h->stats_local_forward_lambda = b; }
    }

    /* :96-122 */
    if (!value_after_tag(f, "COMPO", &buf, &cap, &v)) goto out;
    size_t M = h->model_length;
    h->match_emissions = (float*)calloc(M * NUM_AA, sizeof(float));
    h->insert_emissions = (float*)calloc(M * NUM_AA, sizeof(float));
    h->transitions = (float*)calloc(M * NUM_TR, sizeof(float));
    if (!read_line(f, &buf, &cap)) goto out;
    parse_probs(buf, h->insert_emissions, NUM_AA);
    if (!read_line(f, &buf, &cap)) goto out;
    parse_probs(buf, h->transitions, NUM_TR);
    for (size_t i = 1; i < M; ++i) {
        char tag[32];
        snprintf(tag, sizeof(tag), "%zu", i);
        if (!value_after_tag(f, tag, &buf, &cap, &v)) goto out;
        parse_probs(v, h->match_emissions + i * NUM_AA, NUM_AA);
        if (!read_line(f, &buf, &cap)) goto out;
        parse_probs(buf, h->insert_emissions + i * NUM_AA, NUM_AA);
        if (!read_line(f, &buf, &cap)) goto out;
        parse_probs(buf, h->transitions + i * NUM_TR, NUM_TR);
    }
    rc = 0;
out:
    free(buf);
    fclose(f);
    if (rc) oracle_hmm_free(h);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* MSV (MSV_HMM.hpp:17-44)                                                                    */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    size_t model_length;
    float* emission_scores; /* [20][model_length], residue-major, column 0 = -inf */
    float tr_B_Mk, tr_E_C, tr_E_J;
} oracle_msv;

/* MSV_HMM::MSV_HMM: MSV_HMM.cpp:35-57 */
int oracle_msv_init(const oracle_hmm* h, oracle_msv* m) {
    size_t M = h->model_length;
    m->model_length = M;
    m->emission_scores = (float*)malloc(sizeof(float) * NUM_AA * M);
    if (!m->emission_scores) return -1;
    for (size_t i = 0; i < M; ++i)
        for (size_t j = 0; j < NUM_AA; ++j)
            m->emission_scores[j * M + i] = logf(h->match_emissions[i * NUM_AA + j] / background_frequencies[j]);
    const float nu = 2.0f;
    m->tr_B_Mk = logf(2.0f / (float)(M * (M + 1)));
    m->tr_E_C = logf((nu - 1.0f) / nu);
    m->tr_E_J = logf(1.0f / nu);
    return 0;
}

void oracle_msv_free(oracle_msv* m) {
    free(m->emission_scores);
    m->emission_scores = NULL;
}

/* init_transitions_depend_on_seq: MSV_HMM.cpp:59-64 (L excludes the '#' sentinel) */
void oracle_seq_transitions(size_t L, float* tr_loop, float* tr_move) {
    *tr_loop = logf((float)L / (float)(L + 3));
    *tr_move = logf(3 / (float)(L + 3));
}

/* MSV_HMM::run_on_sequence: MSV_HMM.cpp:74-113 over residue codes 0..19 (no '#').
 * Full (L+1) x (M+5) matrix as in the reference (:86). Returns NAN for a code outside 0..19
 * (the reference throws std::out_of_range from unordered_map::at, :101). */
float oracle_msv_run_codes(const oracle_msv* m, const uint8_t* codes, size_t L) {
    const float ninf = -INFINITY;
    float tr_loop, tr_move;
    oracle_seq_transitions(L, &tr_loop, &tr_move);
    const size_t Mlen = m->model_length;
    const size_t cols = Mlen + 5;
    const size_t E = Mlen, J = Mlen + 1, C = Mlen + 2, N = Mlen + 3, B = Mlen + 4;
    float* dp = (float*)malloc(sizeof(float) * (L + 1) * cols);
    if (!dp) return NAN;
    for (size_t k = 0; k < (L + 1) * cols; ++k) dp[k] = ninf;
    dp[N] = 0.0f;
    dp[B] = tr_move;
    for (size_t i = 1; i <= L; ++i) {
        const unsigned r = codes[i - 1];
        if (r >= NUM_AA) { free(dp); return NAN; }
        const float* e = m->emission_scores + (size_t)r * Mlen;
        const float* prev = dp + (i - 1) * cols;
        float* cur = dp + i * cols;
        for (size_t j = 1; j < Mlen; ++j) {
            const float a = prev[j - 1], b = prev[B] + m->tr_B_Mk;
            cur[j] = e[j] + (a < b ? b : a); /* std::max(a, b) */
            cur[E] = (cur[E] < cur[j]) ? cur[j] : cur[E];
        }
        { const float a = prev[J] + tr_loop, b = cur[E] + m->tr_E_J; cur[J] = (a < b) ? b : a; }
        { const float a = prev[C] + tr_loop, b = cur[E] + m->tr_E_C; cur[C] = (a < b) ? b : a; }
        cur[N] = prev[N] + tr_loop;
        { const float a = cur[N] + tr_move, b = cur[J] + tr_move; cur[B] = (a < b) ? b : a; }
    }
    const float s = dp[L * cols + C] + tr_move;
    free(dp);
    return s;
}

/* Same DP over the reference's Protein_sequence form ('#' + letters). */
float oracle_msv_run_string(const oracle_msv* m, const char* seq) {
    size_t n = strlen(seq);
    if (n == 0) return NAN; /* reference: seq.size()-1 underflows; never produced by its parser */
    size_t L = n - 1;
    uint8_t* codes = (uint8_t*)malloc(L ? L : 1);
    for (size_t i = 0; i < L; ++i) {
        int c = oracle_residue_code(seq[i + 1]);
        codes[i] = (uint8_t)(c < 0 ? 255 : c);
    }
    float s = oracle_msv_run_codes(m, codes, L);
    free(codes);
    return s;
}

/* Score a CSR batch (codes, offsets[n+1]). Single thread, for tests and the port baseline. */
void oracle_msv_run_batch(const oracle_msv* m, const uint8_t* codes, const uint64_t* offsets, size_t n,
                          float* scores) {
    for (size_t s = 0; s < n; ++s)
        scores[s] = oracle_msv_run_codes(m, codes + offsets[s], (size_t)(offsets[s + 1] - offsets[s]));
}

/* ------------------------------------------------------------------------------------------ */
/* Convenience handle API for ctypes                                                          */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    oracle_hmm hmm;
    oracle_msv msv;
} oracle_profile;

oracle_profile* oracle_profile_load(const char* path) {
    oracle_profile* p = (oracle_profile*)calloc(1, sizeof(oracle_profile));
    if (!p) return NULL;
    if (oracle_hmm_load(path, &p->hmm) != 0 || oracle_msv_init(&p->hmm, &p->msv) != 0) {
        oracle_hmm_free(&p->hmm);
        free(p);
        return NULL;
    }
    return p;
}

void oracle_profile_free(oracle_profile* p) {
    if (!p) return;
    oracle_msv_free(&p->msv);
    oracle_hmm_free(&p->hmm);
    free(p);
}

size_t oracle_profile_model_length(const oracle_profile* p) { return p->hmm.model_length; }
const char* oracle_profile_name(const oracle_profile* p) { return p->hmm.name; }
const float* oracle_profile_emission_scores(const oracle_profile* p) { return p->msv.emission_scores; }
const float* oracle_profile_match_emissions(const oracle_profile* p) { return p->hmm.match_emissions; }
const float* oracle_profile_insert_emissions(const oracle_profile* p) { return p->hmm.insert_emissions; }
const float* oracle_profile_transitions(const oracle_profile* p) { return p->hmm.transitions; }
void oracle_profile_constants(const oracle_profile* p, float* out6) {
    out6[0] = p->msv.tr_B_Mk;
    out6[1] = p->msv.tr_E_C;
    out6[2] = p->msv.tr_E_J;
    out6[3] = p->hmm.stats_local_msv_mu;
    out6[4] = p->hmm.stats_local_msv_lambda;
    out6[5] = p->hmm.stats_local_forward_lambda;
}
void oracle_profile_stats(const oracle_profile* p, float* out6) {
    out6[0] = p->hmm.stats_local_msv_mu;
    out6[1] = p->hmm.stats_local_msv_lambda;
    out6[2] = p->hmm.stats_local_viterbi_mu;
    out6[3] = p->hmm.stats_local_viterbi_lambda;
    out6[4] = p->hmm.stats_local_forward_theta;
    out6[5] = p->hmm.stats_local_forward_lambda;
}
float oracle_profile_score_codes(const oracle_profile* p, const uint8_t* codes, size_t L) {
    return oracle_msv_run_codes(&p->msv, codes, L);
}
float oracle_profile_score_string(const oracle_profile* p, const char* seq) {
    return oracle_msv_run_string(&p->msv, seq);
}
void oracle_profile_score_batch(const oracle_profile* p, const uint8_t* codes, const uint64_t* offsets,
                                size_t n, float* scores) {
    oracle_msv_run_batch(&p->msv, codes, offsets, n, scores);
}
