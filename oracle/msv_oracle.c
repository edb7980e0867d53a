/*
 * msv_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C restatement of the reference's MSV CPU path (IvanTyulyandin/HMM_FASTA_Viterbi):
 *   - HMMER3 profile parsing           data_readers/Profile_HMM.cpp:8-122
 *   - FASTA parsing + residue filter   data_readers/FASTA_protein_sequences.cpp:9-44
 *   - MSV host precompute              algorithms/MSV_HMM.cpp:35-57
 *   - per-sequence transitions         algorithms/MSV_HMM.cpp:59-64
 *   - the MSV dynamic programme        algorithms/MSV_HMM.cpp:74-113
 *   - the Viterbi stage over the parse the reference never scores with
 *     (Profile_HMM.cpp:107-120): HMMER3's generic local Viterbi, PARITY UNPINNED (no reference
 *     implementation exists; see the section below)
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
/* Viterbi stage -- PARITY UNPINNED                                           */
/*                                                                                            */
/* The reference parses everything a Viterbi filter needs -- insert_emissions and the 7       */
/* transitions per node (Profile_HMM.hpp:28-29, Profile_HMM.cpp:107-120), STATS LOCAL VITERBI */
/* (Profile_HMM.cpp:86-87) -- and never uses it; there is no reference implementation, and    */
/* HMMER/pyhmmer are absent here.  This is a serial restatement of HMMER3's published generic  */
/* local Viterbi (p7_GViterbi, multihit local mode) over the reference's parse, with the MSV    */
/* path's own specials so the two stages share one null model:                                 */
/*   - match scores  = the MSV table, logf(p / bg) (MSV_HMM.cpp:38-45);                        */
/*   - insert scores = 0 (HMMER3 hardwires them to the background, insert_mode 0), or          */
/*                     logf(ins / bg) of the parsed insert_emissions (insert_mode 1);          */
/*   - transitions   = logf(p) of the parsed probabilities (p = expf(-x), Profile_HMM.cpp:41); */
/*                     only nodes 1 .. LENG-1 are read ('*' entries, which the reference parses */
/*                     as p = 1, sit at node 0 and node LENG and are never read);              */
/*   - B->Mk entry   = tr_B_Mk, E->C = tr_E_C, E->J = tr_E_J, N/C/J loop and move = the        */
/*                     per-length tr_loop / tr_move (MSV_HMM.cpp:49-64);                       */
/*   - exits         = E from every M_k (local) and from D_LENG; I_LENG does not exist.        */
/* Row i, residue r (k = 1 .. LENG, M/I/D(i, 0) = -inf, row 0 all -inf but N = 0, B = move):  */
/*   M(i,k) = max(M(i-1,k-1)+tMM(k-1), I(i-1,k-1)+tIM(k-1), D(i-1,k-1)+tDM(k-1), B(i-1)+tBM)   */
/*            + msc[r][k]                                                                      */
/*   I(i,k) = max(M(i-1,k)+tMI(k), I(i-1,k)+tII(k)) + isc[r][k]            (k < LENG)          */
/*   D(i,k) = max(M(i,k-1)+tMD(k-1), D(i,k-1)+tDD(k-1))                                         */
/*   E = max(max_k M(i,k), D(i,LENG));  J, C, N, B as MSV_HMM.cpp:107-110                      */
/* score = C(L) + move.  Every term is one float add; max is exact, so only the adds matter.   */
/* ------------------------------------------------------------------------------------------ */
enum { T_MM = 0, T_MI = 1, T_MD = 2, T_IM = 3, T_II = 4, T_DM = 5, T_DD = 6 };

typedef struct {
    size_t model_length; /* LENG + 1 */
    float* msc;          /* [20][model_length] match scores (the MSV table) */
    float* isc;          /* [20][model_length] insert scores */
    float* tsc;          /* [model_length][7] log transitions */
    float tr_B_Mk, tr_E_C, tr_E_J;
} oracle_vit;

int oracle_vit_init(const oracle_hmm* h, const oracle_msv* m, int insert_mode, oracle_vit* v) {
    const size_t M = h->model_length;
    memset(v, 0, sizeof(*v));
    v->model_length = M;
    v->msc = (float*)malloc(sizeof(float) * NUM_AA * M);
    v->isc = (float*)malloc(sizeof(float) * NUM_AA * M);
    v->tsc = (float*)malloc(sizeof(float) * NUM_TR * M);
    if (!v->msc || !v->isc || !v->tsc) return -1;
    memcpy(v->msc, m->emission_scores, sizeof(float) * NUM_AA * M);
    for (size_t k = 0; k < M; ++k)
        for (size_t r = 0; r < NUM_AA; ++r)
            v->isc[r * M + k] = insert_mode
                                    ? logf(h->insert_emissions[k * NUM_AA + r] / background_frequencies[r])
                                    : 0.0f;
    for (size_t k = 0; k < M * NUM_TR; ++k) v->tsc[k] = logf(h->transitions[k]);
    v->tr_B_Mk = m->tr_B_Mk;
    v->tr_E_C = m->tr_E_C;
    v->tr_E_J = m->tr_E_J;
    return 0;
}

void oracle_vit_free(oracle_vit* v) {
    free(v->msc);
    free(v->isc);
    free(v->tsc);
    memset(v, 0, sizeof(*v));
}

static float fmax_ref(float a, float b) { return (a < b) ? b : a; } /* std::max(a, b) */

/* Serial generic Viterbi over codes 0..19 (two rolling rows of M, I, D).  NAN for a code >= 20. */
float oracle_vit_run_codes(const oracle_vit* v, const uint8_t* codes, size_t L) {
    const float ninf = -INFINITY;
    float tr_loop, tr_move;
    oracle_seq_transitions(L, &tr_loop, &tr_move);
    const size_t Mlen = v->model_length, K = Mlen - 1; /* K = LENG match states */
    float* buf = (float*)malloc(sizeof(float) * 6 * Mlen);
    if (!buf) return NAN;
    float *pM = buf, *pI = buf + Mlen, *pD = buf + 2 * Mlen;
    float *cM = buf + 3 * Mlen, *cI = buf + 4 * Mlen, *cD = buf + 5 * Mlen;
    for (size_t k = 0; k < 6 * Mlen; ++k) buf[k] = ninf;
    float N = 0.0f, B = tr_move, J = ninf, C = ninf;
    /* t(k, x): transition x out of node k, -inf at node 0 (B enters through tr_B_Mk only) */
#define TSC(k, x) ((k) == 0 ? ninf : v->tsc[(k) * NUM_TR + (x)])
    for (size_t i = 1; i <= L; ++i) {
        const unsigned r = codes[i - 1];
        if (r >= NUM_AA) { free(buf); return NAN; }
        const float* ms = v->msc + (size_t)r * Mlen;
        const float* is = v->isc + (size_t)r * Mlen;
        float E = ninf;
        cM[0] = cI[0] = cD[0] = ninf;
        for (size_t k = 1; k <= K; ++k) {
            float sc = fmax_ref(pM[k - 1] + TSC(k - 1, T_MM), pI[k - 1] + TSC(k - 1, T_IM));
            sc = fmax_ref(sc, pD[k - 1] + TSC(k - 1, T_DM));
            sc = fmax_ref(sc, B + v->tr_B_Mk);
            cM[k] = sc + ms[k];
            E = fmax_ref(E, cM[k]);
            cI[k] = (k < K) ? fmax_ref(pM[k] + TSC(k, T_MI), pI[k] + TSC(k, T_II)) + is[k] : ninf;
            cD[k] = fmax_ref(cM[k - 1] + TSC(k - 1, T_MD), cD[k - 1] + TSC(k - 1, T_DD));
        }
        E = fmax_ref(E, cD[K]);
        J = fmax_ref(J + tr_loop, E + v->tr_E_J);
        C = fmax_ref(C + tr_loop, E + v->tr_E_C);
        N = N + tr_loop;
        B = fmax_ref(N + tr_move, J + tr_move);
        float* t;
        t = pM; pM = cM; cM = t;
        t = pI; pI = cI; cI = t;
        t = pD; pD = cD; cD = t;
    }
#undef TSC
    free(buf);
    return C + tr_move;
}

void oracle_vit_run_batch(const oracle_vit* v, const uint8_t* codes, const uint64_t* offsets, size_t n,
                          float* scores) {
    for (size_t s = 0; s < n; ++s)
        scores[s] = oracle_vit_run_codes(v, codes + offsets[s], (size_t)(offsets[s + 1] - offsets[s]));
}

/* The same DP over caller tables (msc, isc [20][M], tsc [M][7] log transitions; isc NULL = zero): for
 * synthetic models (e.g. transitions that reduce Viterbi to MSV, or near-free D->D chains). */
void oracle_vit_score_tables(const float* msc, const float* isc, const float* tsc, size_t model_length,
                             float tr_B_Mk, float tr_E_C, float tr_E_J, const uint8_t* codes,
                             const uint64_t* offsets, size_t n, float* scores) {
    oracle_vit v;
    v.model_length = model_length;
    v.msc = (float*)msc;
    v.tsc = (float*)tsc;
    v.isc = (float*)calloc(NUM_AA * model_length, sizeof(float));
    if (isc) memcpy(v.isc, isc, sizeof(float) * NUM_AA * model_length);
    v.tr_B_Mk = tr_B_Mk;
    v.tr_E_C = tr_E_C;
    v.tr_E_J = tr_E_J;
    oracle_vit_run_batch(&v, codes, offsets, n, scores);
    free(v.isc);
}

/* ------------------------------------------------------------------------------------------ */
/* Convenience handle API for ctypes                                                          */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    oracle_hmm hmm;
    oracle_msv msv;
    oracle_vit vit[2]; /* insert_mode 0 / 1, built on first use */
    int vit_ready[2];
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
    for (int m = 0; m < 2; ++m)
        if (p->vit_ready[m]) oracle_vit_free(&p->vit[m]);
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

/* Viterbi tables of insert_mode (0 = HMMER3 zero insert scores, 1 = log-odds); not thread-safe on the
 * first call for a mode (call once before scoring from several threads). */
static const oracle_vit* profile_vit(oracle_profile* p, int insert_mode) {
    const int m = insert_mode ? 1 : 0;
    if (!p->vit_ready[m]) {
        if (oracle_vit_init(&p->hmm, &p->msv, m, &p->vit[m]) != 0) return NULL;
        p->vit_ready[m] = 1;
    }
    return &p->vit[m];
}
int oracle_profile_vit_prepare(oracle_profile* p, int insert_mode) { return profile_vit(p, insert_mode) ? 0 : -1; }
void oracle_profile_vit_tables(oracle_profile* p, int insert_mode, float* isc, float* tsc) {
    const oracle_vit* v = profile_vit(p, insert_mode);
    memcpy(isc, v->isc, sizeof(float) * NUM_AA * v->model_length);
    memcpy(tsc, v->tsc, sizeof(float) * NUM_TR * v->model_length);
}
void oracle_profile_vit_score_batch(oracle_profile* p, int insert_mode, const uint8_t* codes,
                                    const uint64_t* offsets, size_t n, float* scores) {
    oracle_vit_run_batch(profile_vit(p, insert_mode), codes, offsets, n, scores);
}
